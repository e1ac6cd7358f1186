"""`ziggy.misc.stats` KL term used by the mean-field model (`stats.py:4-8`)."""
from hipgp_amd.ziggy.hipgp import diag_kl_to_standard  # noqa: F401
