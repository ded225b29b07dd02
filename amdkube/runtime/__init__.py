from .rocshim import RocShim  # noqa: F401
from .hooks import HookService, Hook  # noqa: F401
from .images import ImageStore  # noqa: F401
