from hipgp_amd.ziggy.misc.toeplitz_tensor import *  # noqa: F401,F403
from hipgp_amd.ziggy.misc import toeplitz_tensor as _impl

globals().update({k: v for k, v in vars(_impl).items() if not k.startswith("__")})
