from hipgp_amd.ziggy.hipgp import *  # noqa: F401,F403
from hipgp_amd.ziggy import hipgp as _impl

globals().update({k: v for k, v in vars(_impl).items() if not k.startswith("__")})
