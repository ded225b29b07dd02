from .scheduler import Scheduler, load_policy, PROVIDERS  # noqa: F401
from .cache import SchedulerCache, NodeInfo  # noqa: F401
from .generic import GenericScheduler, FitError  # noqa: F401
from .predicates import PodInfo, PREDICATES, DEFAULT_PREDICATES  # noqa: F401
from .priorities import PRIORITIES, DEFAULT_PRIORITIES  # noqa: F401
from . import extended  # noqa: F401
