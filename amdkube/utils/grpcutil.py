"""gRPC channel helpers for the node-local Unix-socket APIs (device plugins, CRI)."""
from __future__ import annotations

import grpc

# Each channel gets its own subchannel pool. With gRPC's process-global pool, a new channel to a
# socket path that was just closed and re-created (a device plugin or runtime restarting in place)
# reuses the old subchannel, which is still in reconnect backoff, so a 1 s registration dial fails.
UDS_OPTIONS = (("grpc.use_local_subchannel_pool", 1),
               ("grpc.initial_reconnect_backoff_ms", 100),
               ("grpc.max_reconnect_backoff_ms", 1000))


def uds_channel(path: str) -> grpc.aio.Channel:
    return grpc.aio.insecure_channel("unix://" + path, options=UDS_OPTIONS)
