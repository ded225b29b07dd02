from .server import DevicePluginServer, StubDevicePlugin, socket_path  # noqa: F401
from .amd import AMDGPUPlugin, attributes, gpu_type, topology_label, RESOURCE, TOPOLOGY_LABEL  # noqa: F401
