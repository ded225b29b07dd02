from .server import APIServer  # noqa: F401
from .registry import Registry  # noqa: F401
from . import admission  # noqa: F401
