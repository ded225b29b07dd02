"""Container Storage Interface v0.1.0 wire contract (the version the reference's alpha CSI
volume plugin speaks: vendor/github.com/container-storage-interface/spec/lib/go/csi/csi.pb.go).

Field numbers follow csi.pb.go. `VolumeCapability.access_type` is a oneof of `block = 1` and
`mount = 2`; on the wire a oneof is a pair of optional fields, so it is declared flat here
(the runtime proto compiler has no oneof/nesting; the bytes are identical).
"""
from __future__ import annotations

from .compiler import ProtoModule

VERSION = (0, 1, 0)

CSI = ProtoModule("""
syntax = "proto3";
package csi;

service Identity {
  rpc GetSupportedVersions(GetSupportedVersionsRequest) returns (GetSupportedVersionsResponse) {}
  rpc GetPluginInfo(GetPluginInfoRequest) returns (GetPluginInfoResponse) {}
}
service Controller {
  rpc ControllerPublishVolume(ControllerPublishVolumeRequest) returns (ControllerPublishVolumeResponse) {}
  rpc ControllerUnpublishVolume(ControllerUnpublishVolumeRequest) returns (ControllerUnpublishVolumeResponse) {}
  rpc ControllerProbe(ControllerProbeRequest) returns (ControllerProbeResponse) {}
}
service Node {
  rpc NodePublishVolume(NodePublishVolumeRequest) returns (NodePublishVolumeResponse) {}
  rpc NodeUnpublishVolume(NodeUnpublishVolumeRequest) returns (NodeUnpublishVolumeResponse) {}
  rpc GetNodeID(GetNodeIDRequest) returns (GetNodeIDResponse) {}
  rpc NodeProbe(NodeProbeRequest) returns (NodeProbeResponse) {}
}
enum AccessModeMode {
  UNKNOWN = 0;
  SINGLE_NODE_WRITER = 1;
  SINGLE_NODE_READER_ONLY = 2;
  MULTI_NODE_READER_ONLY = 3;
  MULTI_NODE_SINGLE_WRITER = 4;
  MULTI_NODE_MULTI_WRITER = 5;
}
message Version { uint32 major = 1; uint32 minor = 2; uint32 patch = 3; }
message GetSupportedVersionsRequest {}
message GetSupportedVersionsResponse { repeated Version supported_versions = 1; }
message GetPluginInfoRequest { Version version = 1; }
message GetPluginInfoResponse { string name = 1; string vendor_version = 2; map<string, string> manifest = 3; }
message BlockVolume {}
message MountVolume { string fs_type = 1; repeated string mount_flags = 2; }
message AccessMode { AccessModeMode mode = 1; }
message VolumeCapability { BlockVolume block = 1; MountVolume mount = 2; AccessMode access_mode = 3; }
message ControllerPublishVolumeRequest {
  Version version = 1;
  string volume_id = 2;
  string node_id = 3;
  VolumeCapability volume_capability = 4;
  bool readonly = 5;
  map<string, string> user_credentials = 6;
  map<string, string> volume_attributes = 7;
}
message ControllerPublishVolumeResponse { map<string, string> publish_volume_info = 1; }
message ControllerUnpublishVolumeRequest {
  Version version = 1;
  string volume_id = 2;
  string node_id = 3;
  map<string, string> user_credentials = 4;
}
message ControllerUnpublishVolumeResponse {}
message ControllerProbeRequest { Version version = 1; }
message ControllerProbeResponse {}
message NodePublishVolumeRequest {
  Version version = 1;
  string volume_id = 2;
  map<string, string> publish_volume_info = 3;
  string target_path = 4;
  VolumeCapability volume_capability = 5;
  bool readonly = 6;
  map<string, string> user_credentials = 7;
  map<string, string> volume_attributes = 8;
}
message NodePublishVolumeResponse {}
message NodeUnpublishVolumeRequest {
  Version version = 1;
  string volume_id = 2;
  string target_path = 3;
  map<string, string> user_credentials = 4;
}
message NodeUnpublishVolumeResponse {}
message GetNodeIDRequest { Version version = 1; }
message GetNodeIDResponse { string node_id = 1; }
message NodeProbeRequest { Version version = 1; }
message NodeProbeResponse {}
""", "csi/csi.proto")
