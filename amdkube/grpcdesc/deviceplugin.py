"""Device-plugin and plugin-registration wire contracts.

v1alpha2 `deviceplugin` (reference pkg/kubelet/apis/deviceplugin/v1alpha/api.proto:17-154,
constants.go:23-35). `api.pb.go` is the wire authority: GetPluginInfoResponse carries
`map<string,string> labels = 2` (api.pb.go:81-101) although the .proto omits it — included.

`pluginregistration` v1beta Identity service (pkg/kubelet/apis/pluginregistration/v1beta/
api.proto:16-54): served by the plugin, called by the kubelet.

`v1beta1` (upstream Kubernetes Registration/DevicePlugin) — adapter surface so stock
upstream-style plugins (Register → Allocate) can also be consumed.
"""
from __future__ import annotations

from .compiler import ProtoModule

VERSION = "v1alpha2"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"
DEVICE_MANAGER_PATH = "/var/lib/kubelet/device-plugin"
DEVICE_PLUGINS_PATH = DEVICE_MANAGER_PATH + "/plugins"

V1ALPHA2 = ProtoModule("""
syntax = "proto3";
package deviceplugin;

service DevicePlugin {
  rpc GetPluginInfo(GetPluginInfoRequest) returns (GetPluginInfoResponse) {}
  rpc ListAndWatch(ListAndWatchRequest) returns (stream ListAndWatchResponse) {}
  rpc AdmitPod(AdmitPodRequest) returns (AdmitPodResponse) {}
  rpc InitContainer(InitContainerRequest) returns (InitContainerResponse) {}
}
message GetPluginInfoRequest {}
message GetPluginInfoResponse { int64 init_timeout = 1; map<string, string> labels = 2; }
message ListAndWatchRequest {}
message ListAndWatchResponse { repeated Device devices = 1; }
message AdmitPodRequest {
  string pod_name = 1;
  map<string, Container> init_containers = 2;
  map<string, Container> containers = 3;
}
message AdmitPodResponse { PodSpec pod = 1; }
message InitContainerRequest { Container container = 1; }
message InitContainerResponse { ContainerSpec spec = 1; }
message Device { string ID = 1; string health = 2; map<string, string> Attributes = 3; }
message Container { string name = 1; repeated string devices = 2; }
message ContainerSpec {
  map<string, string> envs = 1;
  repeated Mount mounts = 2;
  repeated DeviceSpec devices = 3;
  map<string, string> annotations = 4;
}
message PodSpec { map<string, string> annotations = 1; }
message Mount { string container_path = 1; string host_path = 2; bool read_only = 3; }
message DeviceSpec { string container_path = 1; string host_path = 2; string permissions = 3; }
""", "deviceplugin/v1alpha/api.proto")

REGISTRATION = ProtoModule("""
syntax = "proto3";
package pluginregistration;

service Identity {
  rpc GetSupportedVersions(GetSupportedVersionsRequest) returns (GetSupportedVersionsResponse) {}
  rpc GetPluginIdentity(GetPluginIdentityRequest) returns (GetPluginIdentityResponse) {}
  rpc PluginRegistrationStatus(RegistrationStatus) returns (Empty) {}
}
message Empty {}
message GetSupportedVersionsRequest {}
message GetSupportedVersionsResponse { repeated string supported_versions = 1; }
message GetPluginIdentityRequest { string version = 1; }
message GetPluginIdentityResponse { string resource_name = 1; }
message RegistrationStatus { bool success = 1; string error = 2; }
""", "pluginregistration/v1beta/api.proto")

# Upstream Kubernetes device-plugin API (k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1) —
# the surface BASELINE.json names; served by amdkube's kubelet as an adapter endpoint.
V1BETA1 = ProtoModule("""
syntax = "proto3";
package v1beta1;

service Registration { rpc Register(RegisterRequest) returns (Empty) {} }
service DevicePlugin {
  rpc GetDevicePluginOptions(Empty) returns (DevicePluginOptions) {}
  rpc ListAndWatch(Empty) returns (stream ListAndWatchResponse) {}
  rpc Allocate(AllocateRequest) returns (AllocateResponse) {}
  rpc PreStartContainer(PreStartContainerRequest) returns (PreStartContainerResponse) {}
}
message DevicePluginOptions { bool pre_start_required = 1; bool get_preferred_allocation_available = 2; }
message RegisterRequest { string version = 1; string endpoint = 2; string resource_name = 3; DevicePluginOptions options = 4; }
message Empty {}
message ListAndWatchResponse { repeated Device devices = 1; }
message TopologyInfo { repeated NUMANode nodes = 1; }
message NUMANode { int64 ID = 1; }
message Device { string ID = 1; string health = 2; TopologyInfo topology = 3; }
message PreStartContainerRequest { repeated string devices_ids = 1; }
message PreStartContainerResponse {}
message AllocateRequest { repeated ContainerAllocateRequest container_requests = 1; }
message ContainerAllocateRequest { repeated string devices_ids = 1; }
message AllocateResponse { repeated ContainerAllocateResponse container_responses = 1; }
message ContainerAllocateResponse {
  map<string, string> envs = 1;
  repeated Mount mounts = 2;
  repeated DeviceSpec devices = 3;
  map<string, string> annotations = 4;
}
message Mount { string container_path = 1; string host_path = 2; bool read_only = 3; }
message DeviceSpec { string container_path = 1; string host_path = 2; string permissions = 3; }
""", "deviceplugin/v1beta1/api.proto")

V1BETA1_VERSION = "v1beta1"
KUBELET_SOCKET_V1BETA1 = "/var/lib/kubelet/device-plugins/kubelet.sock"
