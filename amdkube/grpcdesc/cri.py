"""CRI v1alpha1 (package `runtime`) — the subset kubelet ↔ runtime shim needs.

Field numbers follow pkg/kubelet/apis/cri/v1alpha1/runtime/api.proto (services :17-104,
Device :572-582, ContainerConfig :586-645, ContainerStatus :762-797) so that a CRI
client written against that proto interoperates with amdkube's rocshim. Messages not
needed by amdkube (SELinux details, …) are left out; Exec/Attach/PortForward return URLs of
rocshim's streaming server (runtime/streaming.py) as in the reference.
"""
from __future__ import annotations

from .compiler import ProtoModule

CRI = ProtoModule("""
syntax = "proto3";
package runtime;

service RuntimeService {
  rpc Version(VersionRequest) returns (VersionResponse) {}
  rpc RunPodSandbox(RunPodSandboxRequest) returns (RunPodSandboxResponse) {}
  rpc StopPodSandbox(StopPodSandboxRequest) returns (StopPodSandboxResponse) {}
  rpc RemovePodSandbox(RemovePodSandboxRequest) returns (RemovePodSandboxResponse) {}
  rpc PodSandboxStatus(PodSandboxStatusRequest) returns (PodSandboxStatusResponse) {}
  rpc ListPodSandbox(ListPodSandboxRequest) returns (ListPodSandboxResponse) {}
  rpc CreateContainer(CreateContainerRequest) returns (CreateContainerResponse) {}
  rpc StartContainer(StartContainerRequest) returns (StartContainerResponse) {}
  rpc StopContainer(StopContainerRequest) returns (StopContainerResponse) {}
  rpc RemoveContainer(RemoveContainerRequest) returns (RemoveContainerResponse) {}
  rpc ListContainers(ListContainersRequest) returns (ListContainersResponse) {}
  rpc ContainerStatus(ContainerStatusRequest) returns (ContainerStatusResponse) {}
  rpc UpdateContainerResources(UpdateContainerResourcesRequest) returns (UpdateContainerResourcesResponse) {}
  rpc ExecSync(ExecSyncRequest) returns (ExecSyncResponse) {}
  rpc Exec(ExecRequest) returns (ExecResponse) {}
  rpc Attach(AttachRequest) returns (AttachResponse) {}
  rpc PortForward(PortForwardRequest) returns (PortForwardResponse) {}
  rpc ContainerStats(ContainerStatsRequest) returns (ContainerStatsResponse) {}
  rpc ListContainerStats(ListContainerStatsRequest) returns (ListContainerStatsResponse) {}
  rpc UpdateRuntimeConfig(UpdateRuntimeConfigRequest) returns (UpdateRuntimeConfigResponse) {}
  rpc Status(StatusRequest) returns (StatusResponse) {}
  rpc GetContainerEvents(GetEventsRequest) returns (stream ContainerEventResponse) {}
}
service ImageService {
  rpc ListImages(ListImagesRequest) returns (ListImagesResponse) {}
  rpc ImageStatus(ImageStatusRequest) returns (ImageStatusResponse) {}
  rpc PullImage(PullImageRequest) returns (PullImageResponse) {}
  rpc RemoveImage(RemoveImageRequest) returns (RemoveImageResponse) {}
  rpc ImageFsInfo(ImageFsInfoRequest) returns (ImageFsInfoResponse) {}
}

message VersionRequest { string version = 1; }
message VersionResponse { string version = 1; string runtime_name = 2; string runtime_version = 3; string runtime_api_version = 4; }
message DNSConfig { repeated string servers = 1; repeated string searches = 2; repeated string options = 3; }
enum Protocol { TCP = 0; UDP = 1; }
message PortMapping { Protocol protocol = 1; int32 container_port = 2; int32 host_port = 3; string host_ip = 4; }
enum MountPropagation { PROPAGATION_PRIVATE = 0; PROPAGATION_HOST_TO_CONTAINER = 1; PROPAGATION_BIDIRECTIONAL = 2; }
message Mount { string container_path = 1; string host_path = 2; bool readonly = 3; bool selinux_relabel = 4; MountPropagation propagation = 5; }
message NamespaceOption { bool host_network = 1; bool host_pid = 2; bool host_ipc = 3; }
message Int64Value { int64 value = 1; }
message SELinuxOption { string user = 1; string role = 2; string type = 3; string level = 4; }
message LinuxSandboxSecurityContext {
  NamespaceOption namespace_options = 1; SELinuxOption selinux_options = 2; Int64Value run_as_user = 3; bool readonly_rootfs = 4;
  repeated int64 supplemental_groups = 5; bool privileged = 6; string seccomp_profile_path = 7;
}
message LinuxPodSandboxConfig { string cgroup_parent = 1; LinuxSandboxSecurityContext security_context = 2; map<string, string> sysctls = 3; }
message PodSandboxMetadata { string name = 1; string uid = 2; string namespace = 3; uint32 attempt = 4; }
message PodSandboxConfig {
  PodSandboxMetadata metadata = 1; string hostname = 2; string log_directory = 3; DNSConfig dns_config = 4;
  repeated PortMapping port_mappings = 5; map<string, string> labels = 6; map<string, string> annotations = 7;
  LinuxPodSandboxConfig linux = 8;
}
message RunPodSandboxRequest { PodSandboxConfig config = 1; }
message RunPodSandboxResponse { string pod_sandbox_id = 1; }
message StopPodSandboxRequest { string pod_sandbox_id = 1; }
message StopPodSandboxResponse {}
message RemovePodSandboxRequest { string pod_sandbox_id = 1; }
message RemovePodSandboxResponse {}
message PodSandboxStatusRequest { string pod_sandbox_id = 1; bool verbose = 2; }
message PodSandboxNetworkStatus { string ip = 1; }
message Namespace { NamespaceOption options = 2; }
message LinuxPodSandboxStatus { Namespace namespaces = 1; }
enum PodSandboxState { SANDBOX_READY = 0; SANDBOX_NOTREADY = 1; }
message PodSandboxStatus {
  string id = 1; PodSandboxMetadata metadata = 2; PodSandboxState state = 3; int64 created_at = 4;
  PodSandboxNetworkStatus network = 5; LinuxPodSandboxStatus linux = 6; map<string, string> labels = 7;
  map<string, string> annotations = 8;
}
message PodSandboxStatusResponse { PodSandboxStatus status = 1; map<string, string> info = 2; }
message PodSandboxStateValue { PodSandboxState state = 1; }
message PodSandboxFilter { string id = 1; PodSandboxStateValue state = 2; map<string, string> label_selector = 3; }
message ListPodSandboxRequest { PodSandboxFilter filter = 1; }
message PodSandbox {
  string id = 1; PodSandboxMetadata metadata = 2; PodSandboxState state = 3; int64 created_at = 4;
  map<string, string> labels = 5; map<string, string> annotations = 6;
}
message ListPodSandboxResponse { repeated PodSandbox items = 1; }
message ImageSpec { string image = 1; }
message KeyValue { string key = 1; string value = 2; }
message LinuxContainerResources {
  int64 cpu_period = 1; int64 cpu_quota = 2; int64 cpu_shares = 3; int64 memory_limit_in_bytes = 4;
  int64 oom_score_adj = 5; string cpuset_cpus = 6; string cpuset_mems = 7;
}
message Capability { repeated string add_capabilities = 1; repeated string drop_capabilities = 2; }
message LinuxContainerSecurityContext {
  Capability capabilities = 1; bool privileged = 2; NamespaceOption namespace_options = 3; SELinuxOption selinux_options = 4;
  Int64Value run_as_user = 5; string run_as_username = 6; bool readonly_rootfs = 7;
  repeated int64 supplemental_groups = 8; string apparmor_profile = 9; string seccomp_profile_path = 10; bool no_new_privs = 11;
}
message LinuxContainerConfig { LinuxContainerResources resources = 1; LinuxContainerSecurityContext security_context = 2; }
message ContainerMetadata { string name = 1; uint32 attempt = 2; }
message Device { string container_path = 1; string host_path = 2; string permissions = 3; }
message ContainerConfig {
  ContainerMetadata metadata = 1; ImageSpec image = 2; repeated string command = 3; repeated string args = 4;
  string working_dir = 5; repeated KeyValue envs = 6; repeated Mount mounts = 7; repeated Device devices = 8;
  map<string, string> labels = 9; map<string, string> annotations = 10; string log_path = 11;
  bool stdin = 12; bool stdin_once = 13; bool tty = 14; LinuxContainerConfig linux = 15;
}
message CreateContainerRequest { string pod_sandbox_id = 1; ContainerConfig config = 2; PodSandboxConfig sandbox_config = 3; }
message CreateContainerResponse { string container_id = 1; }
message StartContainerRequest { string container_id = 1; }
message StartContainerResponse {}
message StopContainerRequest { string container_id = 1; int64 timeout = 2; }
message StopContainerResponse {}
message RemoveContainerRequest { string container_id = 1; }
message RemoveContainerResponse {}
enum ContainerState { CONTAINER_CREATED = 0; CONTAINER_RUNNING = 1; CONTAINER_EXITED = 2; CONTAINER_UNKNOWN = 3; }
message ContainerStateValue { ContainerState state = 1; }
message ContainerFilter { string id = 1; ContainerStateValue state = 2; string pod_sandbox_id = 3; map<string, string> label_selector = 4; }
message ListContainersRequest { ContainerFilter filter = 1; }
message Container {
  string id = 1; string pod_sandbox_id = 2; ContainerMetadata metadata = 3; ImageSpec image = 4; string image_ref = 5;
  ContainerState state = 6; int64 created_at = 7; map<string, string> labels = 8; map<string, string> annotations = 9;
}
message ListContainersResponse { repeated Container containers = 1; }
message ContainerStatusRequest { string container_id = 1; bool verbose = 2; }
message ContainerStatus {
  string id = 1; ContainerMetadata metadata = 2; ContainerState state = 3; int64 created_at = 4; int64 started_at = 5;
  int64 finished_at = 6; int32 exit_code = 7; ImageSpec image = 8; string image_ref = 9; string reason = 10;
  string message = 11; map<string, string> labels = 12; map<string, string> annotations = 13; repeated Mount mounts = 14;
  string log_path = 15;
}
message ContainerStatusResponse { ContainerStatus status = 1; map<string, string> info = 2; }
message UpdateContainerResourcesRequest { string container_id = 1; LinuxContainerResources linux = 2; }
message UpdateContainerResourcesResponse {}
message ExecSyncRequest { string container_id = 1; repeated string cmd = 2; int64 timeout = 3; }
message ExecSyncResponse { bytes stdout = 1; bytes stderr = 2; int32 exit_code = 3; }
message ExecRequest { string container_id = 1; repeated string cmd = 2; bool tty = 3; bool stdin = 4; bool stdout = 5; bool stderr = 6; }
message ExecResponse { string url = 1; }
message AttachRequest { string container_id = 1; bool stdin = 2; bool tty = 3; bool stdout = 4; bool stderr = 5; }
message AttachResponse { string url = 1; }
message PortForwardRequest { string pod_sandbox_id = 1; repeated int32 port = 2; }
message PortForwardResponse { string url = 1; }
message ImageFilter { ImageSpec image = 1; }
message ListImagesRequest { ImageFilter filter = 1; }
message Image { string id = 1; repeated string repo_tags = 2; repeated string repo_digests = 3; uint64 size = 4; Int64Value uid = 5; string username = 6; }
message ListImagesResponse { repeated Image images = 1; }
message ImageStatusRequest { ImageSpec image = 1; bool verbose = 2; }
message ImageStatusResponse { Image image = 1; map<string, string> info = 2; }
message AuthConfig { string username = 1; string password = 2; string auth = 3; string server_address = 4; string identity_token = 5; string registry_token = 6; }
message PullImageRequest { ImageSpec image = 1; AuthConfig auth = 2; PodSandboxConfig sandbox_config = 3; }
message PullImageResponse { string image_ref = 1; }
message RemoveImageRequest { ImageSpec image = 1; }
message RemoveImageResponse {}
message NetworkConfig { string pod_cidr = 1; }
message RuntimeConfig { NetworkConfig network_config = 1; }
message UpdateRuntimeConfigRequest { RuntimeConfig runtime_config = 1; }
message UpdateRuntimeConfigResponse {}
message RuntimeCondition { string type = 1; bool status = 2; string reason = 3; string message = 4; }
message RuntimeStatus { repeated RuntimeCondition conditions = 1; }
message StatusRequest { bool verbose = 1; }
message StatusResponse { RuntimeStatus status = 1; map<string, string> info = 2; }
message ImageFsInfoRequest {}
message UInt64Value { uint64 value = 1; }
message StorageIdentifier { string uuid = 1; }
message FilesystemUsage { int64 timestamp = 1; StorageIdentifier storage_id = 2; UInt64Value used_bytes = 3; UInt64Value inodes_used = 4; }
message ImageFsInfoResponse { repeated FilesystemUsage image_filesystems = 1; }
message ContainerStatsRequest { string container_id = 1; }
message ContainerStatsResponse { ContainerStats stats = 1; }
message ContainerStatsFilter { string id = 1; string pod_sandbox_id = 2; map<string, string> label_selector = 3; }
message ListContainerStatsRequest { ContainerStatsFilter filter = 1; }
message ListContainerStatsResponse { repeated ContainerStats stats = 1; }
message ContainerAttributes { string id = 1; ContainerMetadata metadata = 2; map<string, string> labels = 3; map<string, string> annotations = 4; }
message ContainerStats { ContainerAttributes attributes = 1; CpuUsage cpu = 2; MemoryUsage memory = 3; FilesystemUsage writable_layer = 4; }
message CpuUsage { int64 timestamp = 1; UInt64Value usage_core_nano_seconds = 2; }
message MemoryUsage {
  int64 timestamp = 1; UInt64Value working_set_bytes = 2;
  // later CRI revisions' additions, same field numbers (older peers ignore them)
  UInt64Value available_bytes = 3; UInt64Value usage_bytes = 4; UInt64Value rss_bytes = 5;
  UInt64Value page_faults = 6; UInt64Value major_page_faults = 7;
}
message GetEventsRequest {}
enum ContainerEventType { CONTAINER_CREATED_EVENT = 0; CONTAINER_STARTED_EVENT = 1; CONTAINER_STOPPED_EVENT = 2; CONTAINER_DELETED_EVENT = 3; }
message ContainerEventResponse {
  string container_id = 1; ContainerEventType container_event_type = 2; int64 created_at = 3;
  PodSandboxStatus pod_sandbox_status = 4; repeated ContainerStatus containers_statuses = 5;
}
""", "runtime/v1alpha1/api.proto")
# GetContainerEvents is the evented-PLEG stream of later CRI versions (KEP-3386) back-ported
# into amdkube's CRI: the kubelet learns about container starts/exits immediately instead of
# waiting for the next relist (the relist still runs as the consistency backstop).

API_VERSION = "0.1.0"
# trailing-metadata key of rocshim's mutating calls: "<sandbox id>:<created_at>" of the newest
# event emitted for the call's sandbox when it returned ("" = no event to wait for)
EVENT_TRAILER = "amdkube-event"
