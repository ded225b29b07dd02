from .rest import Client, ChaosError  # noqa: F401
from .informer import Informer, SharedInformerFactory, ResourceEventHandler  # noqa: F401
from .workqueue import WorkQueue, RateLimitingQueue, DelayingQueue, parallelize  # noqa: F401
from .leaderelection import LeaderElector  # noqa: F401
from .record import EventRecorder  # noqa: F401
