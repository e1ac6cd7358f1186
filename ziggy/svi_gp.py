"""`ziggy.svi_gp` names the hot-path models use (the SVI fit driver itself is out of scope)."""
from hipgp_amd.ziggy.hipgp import SviGP  # noqa: F401
