from .mvcc import MVCCStore, KV, Event, Compacted, CASFailed, KeyExists, KeyNotFound, PUT, DELETE  # noqa: F401
from .storage import Storage, Filter, FilteredWatch, event_object  # noqa: F401
