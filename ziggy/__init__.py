"""Drop-in `ziggy` namespace: re-exports the MI355X implementation in hipgp_amd.ziggy so
code written against the reference (`from ziggy.misc.toeplitz_tensor import ToeplitzTensor`)
runs unchanged on the HIP path."""
