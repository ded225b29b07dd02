"""DeviceManager state: per-endpoint device store, endpoint store, node capacity store and
the pod-annotation cache.

Reference (pkg/kubelet/cm/devicemanager/):
  device_store.go:25-37,86-121   Update(devs) → (added, updated, deleted); health flip =
                                 updated. Deliberate fix #11: attribute changes also count
                                 as updated (the reference ignores them, :103-105).
  device_store.go:157-183        alwaysEmptyDeviceStore null object.
  endpoint_handler.go:204-248    endpoint store: Endpoint/SwapEndpoint/DeleteEndpoint.
  manager_store.go:29-130        ExtendedResourceMap; drop a resource when its domain empties
                                 and report it in `removed`; GetCapacity deep-copies + clears
                                 removed; HasDevices = exists and Healthy.
  cache.go:26-100                pod UID → RunPodOptions{Annotations} from AdmitPod. Deliberate
                                 fix #3: nothing is cached for a failed/empty AdmitPod.
"""
from __future__ import annotations

import copy
import threading

from ...grpcdesc.deviceplugin import HEALTHY


def _dev(d) -> dict:
    if isinstance(d, dict):
        return {"ID": d["ID"], "health": d.get("health", HEALTHY), "Attributes": dict(d.get("Attributes") or {})}
    return {"ID": d.ID, "health": d.health or HEALTHY, "Attributes": dict(d.Attributes)}


class DeviceStore:
    def __init__(self):
        self._lock = threading.Lock()
        self.devices: dict[str, dict] = {}

    def update(self, devs) -> tuple[list[dict], list[dict], list[dict]]:
        new = {d["ID"]: d for d in (_dev(x) for x in devs)}
        added, updated, deleted = [], [], []
        with self._lock:
            for did, d in new.items():
                cur = self.devices.get(did)
                if cur is None:
                    added.append(d)
                elif cur["health"] != d["health"] or cur["Attributes"] != d["Attributes"]:
                    updated.append(d)
            for did, d in self.devices.items():
                if did not in new:
                    deleted.append(d)
            self.devices = new
        return added, updated, deleted

    def devs(self) -> list[dict]:
        with self._lock:
            return [dict(d) for d in self.devices.values()]

    def healthy(self) -> list[dict]:
        return [d for d in self.devs() if d["health"] == HEALTHY]


class AlwaysEmptyDeviceStore(DeviceStore):
    def update(self, devs):
        return [], [], []

    def devs(self):
        return []


class EndpointStore:
    def __init__(self):
        self._lock = threading.Lock()
        self.endpoints: dict[str, object] = {}

    def endpoint(self, rname):
        with self._lock:
            return self.endpoints.get(rname)

    def swap_endpoint(self, e):
        with self._lock:
            old = self.endpoints.get(e.resource_name)
            self.endpoints[e.resource_name] = e
            return old

    def delete_endpoint(self, rname, only_if=None) -> bool:
        with self._lock:
            cur = self.endpoints.get(rname)
            if cur is None or (only_if is not None and cur is not only_if):
                return False
            del self.endpoints[rname]
            return True

    def all(self):
        with self._lock:
            return dict(self.endpoints)


class ManagerStore:
    """Node-level view: {resource: {"resources": {id: {id, health, attributes}}}}."""

    def __init__(self):
        self._lock = threading.Lock()
        self.capacity: dict[str, dict] = {}
        self.removed: list[str] = []
        self.version = 0
        self.listeners = []

    def update_capacity(self, rname: str, added, updated, deleted):
        with self._lock:
            dom = self.capacity.setdefault(rname, {"resources": {}})
            for d in list(added) + list(updated):
                dom["resources"][d["ID"]] = {"id": d["ID"], "health": d["health"], "attributes": dict(d["Attributes"])}
            for d in deleted:
                dom["resources"].pop(d["ID"], None)
            if not dom["resources"]:
                del self.capacity[rname]
                if rname not in self.removed:
                    self.removed.append(rname)
            elif rname in self.removed:
                self.removed.remove(rname)
            self.version += 1
        for cb in list(self.listeners):
            cb(rname)

    def get_capacity(self) -> tuple[dict, list[str]]:
        with self._lock:
            cap = copy.deepcopy(self.capacity)
            removed, self.removed = self.removed, []
            return cap, removed

    def peek(self) -> dict:
        with self._lock:
            return copy.deepcopy(self.capacity)

    def has_devices(self, rname: str, ids) -> tuple[bool, str]:
        with self._lock:
            dom = self.capacity.get(rname)
            if dom is None:
                return False, f"resource {rname} is not available on this node"
            for did in ids:
                d = dom["resources"].get(did)
                if d is None:
                    return False, f"device {did} of {rname} does not exist"
                if d["health"] != HEALTHY:
                    return False, f"device {did} of {rname} is unhealthy"
            return True, ""


class PodResourceCache:
    def __init__(self):
        self._lock = threading.Lock()
        self.pods: dict[str, dict] = {}

    def cache(self, uid: str, annotations: dict | None):
        if not annotations:
            return
        with self._lock:
            self.pods.setdefault(uid, {}).update(annotations)

    def get(self, uid: str) -> dict:
        with self._lock:
            return dict(self.pods.get(uid, {}))

    def delete(self, uid: str):
        with self._lock:
            self.pods.pop(uid, None)

    def uids(self):
        with self._lock:
            return list(self.pods)
