"""`ziggy.misc` overlay: hot-path modules from hipgp_amd (see ziggy/__init__.py), the rest
from the next `ziggy/misc` on sys.path."""
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)
