"""hipgp_amd — MI355X-native (gfx950) structured-kernel PCG hot path of HIP-GP.

`hipgp_amd.ziggy` mirrors the reference `ziggy` package's operator API for this path
(ToeplitzTensor, conj_grad/conj_grad2, ToeplitzMatmul/gram_solve, InvMatmul, kernels);
the top-level `ziggy` package re-exports it so experiment code imports it unchanged.
"""
__version__ = "0.1.0"
