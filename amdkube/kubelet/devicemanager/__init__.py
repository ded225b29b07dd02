from .manager import ManagerImpl, ManagerStub, AdmissionError, container_device_requests  # noqa: F401
from .watcher import PluginWatcher  # noqa: F401
from .stores import DeviceStore, AlwaysEmptyDeviceStore, EndpointStore, ManagerStore, PodResourceCache  # noqa: F401
from .endpoint import Endpoint, EndpointHandler, Validator, RegistrationError  # noqa: F401
from .run_options import merge_container_specs  # noqa: F401
