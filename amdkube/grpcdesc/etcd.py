"""etcd v3 client API (the subset the apiserver's storage uses) as a runtime-built gRPC module.

Reference: vendor/github.com/coreos/etcd/etcdserver/etcdserverpb/rpc.proto (KV, Watch, Lease,
Maintenance.Status) and vendor/github.com/coreos/etcd/mvcc/mvccpb/kv.proto (KeyValue, Event),
driven by staging/src/k8s.io/apiserver/pkg/storage/etcd3/{store,watcher,compact}.go. Every
message below carries ALL of the reference message's fields with the reference numbers and
types (tests/test_etcd.py compares against the `fileDescriptorRpc` / `fileDescriptorKv` blobs
extracted into tests/fixtures/reference_descriptors). KeyValue and Event live in this one
package here (mvccpb upstream): a package name never reaches the wire, gRPC method paths
(`/etcdserverpb.KV/Txn`) do and match.
"""
from __future__ import annotations

from .compiler import ProtoModule

ETCD = ProtoModule("""
syntax = "proto3";
package etcdserverpb;

service KV {
  rpc Range(RangeRequest) returns (RangeResponse) {}
  rpc Put(PutRequest) returns (PutResponse) {}
  rpc DeleteRange(DeleteRangeRequest) returns (DeleteRangeResponse) {}
  rpc Txn(TxnRequest) returns (TxnResponse) {}
  rpc Compact(CompactionRequest) returns (CompactionResponse) {}
}
service Watch {
  rpc Watch(stream WatchRequest) returns (stream WatchResponse) {}
}
service Lease {
  rpc LeaseGrant(LeaseGrantRequest) returns (LeaseGrantResponse) {}
  rpc LeaseRevoke(LeaseRevokeRequest) returns (LeaseRevokeResponse) {}
  rpc LeaseKeepAlive(stream LeaseKeepAliveRequest) returns (stream LeaseKeepAliveResponse) {}
}
service Maintenance {
  rpc Status(StatusRequest) returns (StatusResponse) {}
}

message KeyValue {
  bytes key = 1;
  int64 create_revision = 2;
  int64 mod_revision = 3;
  int64 version = 4;
  bytes value = 5;
  int64 lease = 6;
}
message Event {
  enum EventType { PUT = 0; DELETE = 1; }
  EventType type = 1;
  KeyValue kv = 2;
  KeyValue prev_kv = 3;
}

message ResponseHeader { uint64 cluster_id = 1; uint64 member_id = 2; int64 revision = 3; uint64 raft_term = 4; }

message RangeRequest {
  enum SortOrder { NONE = 0; ASCEND = 1; DESCEND = 2; }
  enum SortTarget { KEY = 0; VERSION = 1; CREATE = 2; MOD = 3; VALUE = 4; }
  bytes key = 1;
  bytes range_end = 2;
  int64 limit = 3;
  int64 revision = 4;
  SortOrder sort_order = 5;
  SortTarget sort_target = 6;
  bool serializable = 7;
  bool keys_only = 8;
  bool count_only = 9;
  int64 min_mod_revision = 10;
  int64 max_mod_revision = 11;
  int64 min_create_revision = 12;
  int64 max_create_revision = 13;
}
message RangeResponse { ResponseHeader header = 1; repeated mvccpb.KeyValue kvs = 2; bool more = 3; int64 count = 4; }

message PutRequest { bytes key = 1; bytes value = 2; int64 lease = 3; bool prev_kv = 4; }
message PutResponse { ResponseHeader header = 1; mvccpb.KeyValue prev_kv = 2; }

message DeleteRangeRequest { bytes key = 1; bytes range_end = 2; bool prev_kv = 3; }
message DeleteRangeResponse { ResponseHeader header = 1; int64 deleted = 2; repeated mvccpb.KeyValue prev_kvs = 3; }

message RequestOp {
  oneof request {
    RangeRequest request_range = 1;
    PutRequest request_put = 2;
    DeleteRangeRequest request_delete_range = 3;
  }
}
message ResponseOp {
  oneof response {
    RangeResponse response_range = 1;
    PutResponse response_put = 2;
    DeleteRangeResponse response_delete_range = 3;
  }
}
message Compare {
  enum CompareResult { EQUAL = 0; GREATER = 1; LESS = 2; NOT_EQUAL = 3; }
  enum CompareTarget { VERSION = 0; CREATE = 1; MOD = 2; VALUE = 3; }
  CompareResult result = 1;
  CompareTarget target = 2;
  bytes key = 3;
  oneof target_union {
    int64 version = 4;
    int64 create_revision = 5;
    int64 mod_revision = 6;
    bytes value = 7;
  }
}
message TxnRequest { repeated Compare compare = 1; repeated RequestOp success = 2; repeated RequestOp failure = 3; }
message TxnResponse { ResponseHeader header = 1; bool succeeded = 2; repeated ResponseOp responses = 3; }

message CompactionRequest { int64 revision = 1; bool physical = 2; }
message CompactionResponse { ResponseHeader header = 1; }

message WatchRequest {
  oneof request_union {
    WatchCreateRequest create_request = 1;
    WatchCancelRequest cancel_request = 2;
  }
}
message WatchCreateRequest {
  enum FilterType { NOPUT = 0; NODELETE = 1; }
  bytes key = 1;
  bytes range_end = 2;
  int64 start_revision = 3;
  bool progress_notify = 4;
  repeated FilterType filters = 5;
  bool prev_kv = 6;
}
message WatchCancelRequest { int64 watch_id = 1; }
message WatchResponse {
  ResponseHeader header = 1;
  int64 watch_id = 2;
  bool created = 3;
  bool canceled = 4;
  int64 compact_revision = 5;
  repeated mvccpb.Event events = 11;
}

message LeaseGrantRequest { int64 TTL = 1; int64 ID = 2; }
message LeaseGrantResponse { ResponseHeader header = 1; int64 ID = 2; int64 TTL = 3; string error = 4; }
message LeaseRevokeRequest { int64 ID = 1; }
message LeaseRevokeResponse { ResponseHeader header = 1; }
message LeaseKeepAliveRequest { int64 ID = 1; }
message LeaseKeepAliveResponse { ResponseHeader header = 1; int64 ID = 2; int64 TTL = 3; }

message StatusRequest {}
message StatusResponse {
  ResponseHeader header = 1;
  string version = 2;
  int64 dbSize = 3;
  uint64 leader = 4;
  uint64 raftIndex = 5;
  uint64 raftTerm = 6;
}
""", "etcdserverpb/rpc.proto")

# the reference's etcd3 store compares/targets by these numbers (rpc.proto Compare enums)
EQUAL, GREATER, LESS, NOT_EQUAL = 0, 1, 2, 3
T_VERSION, T_CREATE, T_MOD, T_VALUE = 0, 1, 2, 3
EV_PUT, EV_DELETE = 0, 1
