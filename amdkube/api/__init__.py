"""amdkube API machinery: object model, selectors, quantities, validation, defaulting.

Importing this package registers the defaulting/validation hooks on SCHEME.
"""
from . import defaults as _defaults  # noqa: F401  (registers hooks)
from . import validation as _validation  # noqa: F401
from . import extgroups as _extgroups  # noqa: F401
from .scheme import SCHEME, ResourceInfo, encode, decode, load_manifests, dump_yaml  # noqa: F401
from .meta import StatusError  # noqa: F401
from .quantity import Quantity  # noqa: F401
