from hipgp_amd.ziggy.misc._inv_matmul import *  # noqa: F401,F403
from hipgp_amd.ziggy.misc import _inv_matmul as _impl

globals().update({k: v for k, v in vars(_impl).items() if not k.startswith("__")})
