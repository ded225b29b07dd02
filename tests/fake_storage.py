"""In-memory fakes of four vendor storage APIs for tests/test_vendor_volumes.py: the Flocker
control service (datasets move to a new primary after one state poll), StorageOS (basic auth,
volumes with device files written under a fake /var/lib/storageos/volumes), the openstorage
(Portworx) REST API and the ScaleIO gateway (login token, SDC mapping; a mapped volume's
emc-vol device appears under a fake /dev/disk/by-id). Shapes follow public API documentation;
no real backend exists offline."""
from __future__ import annotations

import base64
import os
import uuid

from tests.fake_smallclouds import _Server

J = "application/json"


class FakeFlocker(_Server):
    def __init__(self, nodes: dict[str, str]):
        self.nodes = {u: h for u, h in nodes.items()}          # uuid -> host ip
        self.config: dict[str, dict] = {}
        self.state: dict[str, dict] = {}
        self.moves: list[tuple] = []
        self._serve(self._handle)

    def add_dataset(self, name, primary):
        ds = str(uuid.uuid4())
        self.config[ds] = {"dataset_id": ds, "primary": primary, "metadata": {"name": name}, "deleted": False}
        self.state[ds] = {"dataset_id": ds, "primary": primary, "path": f"/flocker/{ds}"}
        return ds

    def _handle(self, method, path, q, body, headers):
        with self.lock:
            if path == "/v1/state/nodes":
                return 200, J, [{"uuid": u, "host": h} for u, h in self.nodes.items()]
            if path == "/v1/state/datasets":
                out = list(self.state.values())
                for ds, c in self.config.items():            # a pending move lands on the next poll
                    st = self.state.get(ds)
                    if st is None or st["primary"] != c["primary"]:
                        self.state[ds] = {"dataset_id": ds, "primary": c["primary"], "path": f"/flocker/{ds}"}
                return 200, J, out
            if path == "/v1/configuration/datasets" and method == "GET":
                return 200, J, list(self.config.values())
            if path == "/v1/configuration/datasets" and method == "POST":
                ds = str(uuid.uuid4())
                self.config[ds] = {"dataset_id": ds, "primary": body["primary"], "metadata": body.get("metadata") or {},
                                   "maximum_size": body.get("maximum_size"), "deleted": False}
                return 201, J, self.config[ds]
            ds = path.rsplit("/", 1)[-1]
            if ds not in self.config:
                return 404, J, {"description": "Dataset not found."}
            if method == "POST":
                self.config[ds]["primary"] = body["primary"]
                self.moves.append((ds, body["primary"]))
                return 200, J, self.config[ds]
            if method == "DELETE":
                self.config.pop(ds)
                self.state.pop(ds, None)
                return 200, J, {"dataset_id": ds}
        return 404, J, {}


class FakeStorageOS(_Server):
    def __init__(self, dev_dir: str, user="storageos", password="storageos"):
        self.dev_dir, self.auth = dev_dir, "Basic " + base64.b64encode(f"{user}:{password}".encode()).decode()
        self.volumes: dict[tuple, dict] = {}
        self.mounts: dict[tuple, dict] = {}
        self._serve(self._handle)

    def add_volume(self, ns, name, size=5, file_backed=True):
        vid = str(uuid.uuid4())
        self.volumes[(ns, name)] = {"id": vid, "name": name, "namespace": ns, "size": size, "fsType": "ext4"}
        os.makedirs(self.dev_dir, exist_ok=True)
        p = os.path.join(self.dev_dir, vid)
        if file_backed:
            open(p, "wb").close()
        else:
            os.makedirs(p)       # stands in for a block device node (not a regular file)
        return vid

    def _handle(self, method, path, q, body, headers):
        if headers.get("Authorization") != self.auth:
            return 401, J, {"message": "unauthorized"}
        seg = path.strip("/").split("/")               # v1 namespaces ns volumes [name [mount|unmount]]
        if seg[:2] != ["v1", "namespaces"] or len(seg) < 4 or seg[3] != "volumes":
            return 404, J, {}
        ns = seg[2]
        with self.lock:
            if len(seg) == 4 and method == "POST":
                v = {"id": str(uuid.uuid4()), "name": body["name"], "namespace": ns, "size": body["size"], "pool": body.get("pool"),
                     "fsType": body.get("fsType"), "labels": body.get("labels")}
                self.volumes[(ns, body["name"])] = v
                return 201, J, v
            key = (ns, seg[4])
            if key not in self.volumes:
                return 404, J, {"message": "volume not found"}
            if len(seg) == 5 and method == "GET":
                return 200, J, self.volumes[key]
            if len(seg) == 5 and method == "DELETE":
                del self.volumes[key]
                return 200, J, {}
            if seg[5] == "mount":
                self.mounts[key] = body
            elif seg[5] == "unmount":
                self.mounts.pop(key, None)
            return 200, J, {}


class FakePortworx(_Server):
    def __init__(self):
        self.vols: dict[str, dict] = {}
        self.actions: list[tuple] = []
        self._serve(self._handle)

    def add_volume(self, name, size=1 << 30):
        vid = str(uuid.uuid4().int)[:18]
        self.vols[vid] = {"id": vid, "locator": {"name": name}, "spec": {"size": size}, "attached_on": "", "attach_path": []}
        return vid

    def _handle(self, method, path, q, body, headers):
        with self.lock:
            rest = path[len("/v1/osd-volumes"):].strip("/")
            if not rest and method == "POST":
                vid = str(uuid.uuid4().int)[:18]
                self.vols[vid] = {"id": vid, "locator": body["locator"], "spec": body["spec"], "attached_on": "", "attach_path": []}
                return 200, J, {"id": vid}
            v = self.vols.get(rest)
            if v is None:
                return (200, J, []) if method == "GET" else (404, J, {"error": f"volume {rest} not found"})
            if method == "GET":
                return 200, J, [v]
            if method == "DELETE":
                if v["attached_on"]:
                    return 200, J, {"error": "volume is attached"}
                del self.vols[rest]
                return 200, J, {}
            a = body["action"]
            self.actions.append((rest, dict(a)))
            if a.get("attach") == 1:
                v["attached_on"] = "node-a"
                return 200, J, {"device_path": f"/dev/pxd/pxd{rest}"}
            if a.get("attach") == 2:
                if v["attach_path"]:
                    return 200, J, {"error": "volume is mounted"}
                v["attached_on"] = ""
            if a.get("mount") == 1:
                if not v["attached_on"]:
                    return 200, J, {"error": "volume is not attached"}
                v["attach_path"].append(a["mount_path"])
            if a.get("mount") == 2:
                v["attach_path"] = [p for p in v["attach_path"] if p != a["mount_path"]]
            return 200, J, {}


class FakeScaleIO(_Server):
    USER, PASSWORD, MDM = "sio-admin", "sio-pw", "788d9efb0a8f20cb"

    def __init__(self, by_id_dir: str, sdc_guid: str):
        self.by_id = by_id_dir
        self.token = uuid.uuid4().hex
        self.sdcs = {"sdc-1": sdc_guid, "sdc-2": "OTHER-GUID"}
        self.volumes: dict[str, dict] = {}
        self._serve(self._handle)

    def add_volume(self, name, kb=8 << 20):
        vid = uuid.uuid4().hex[:16]
        self.volumes[vid] = {"id": vid, "name": name, "sizeInKb": kb, "mappedSdcInfo": []}
        return vid

    def _dev(self, vid):
        return os.path.join(self.by_id, f"emc-vol-{self.MDM}-{vid}")

    def _handle(self, method, path, q, body, headers):
        if path == "/api/login":
            want = "Basic " + base64.b64encode(f"{self.USER}:{self.PASSWORD}".encode()).decode()
            return (200, J, f'"{self.token}"') if headers.get("Authorization") == want else (401, J, {"message": "bad login"})
        if headers.get("Authorization") != "Basic " + base64.b64encode(f"{self.USER}:{self.token}".encode()).decode():
            return 401, J, {"message": "token"}
        p = path[len("/api"):]
        with self.lock:
            if p == "/types/System/instances":
                return 200, J, [{"id": "sys-1", "name": "sio-sys"}]
            if p == "/instances/System::sys-1/relationships/ProtectionDomain":
                return 200, J, [{"id": "pd-1", "name": "pd-gpu"}]
            if p == "/instances/ProtectionDomain::pd-1/relationships/StoragePool":
                return 200, J, [{"id": "sp-1", "name": "sp-ssd"}]
            if p == "/types/Sdc/instances":
                return 200, J, [{"id": i, "sdcGuid": g} for i, g in self.sdcs.items()]
            if p == "/types/Volume/instances/action/queryIdByKey":
                vid = next((v["id"] for v in self.volumes.values() if v["name"] == body["name"]), None)
                return (200, J, f'"{vid}"') if vid else (500, J, {"message": "Could not find the volume"})
            if p == "/types/Volume/instances":
                vid = self.add_volume(body["name"], int(body["volumeSizeInKb"]))
                self.volumes[vid].update(storagePoolId=body["storagePoolId"], volumeType=body["volumeType"])
                return 200, J, {"id": vid}
            vid = p.split("::", 1)[-1].split("/", 1)[0]
            v = self.volumes.get(vid)
            if v is None:
                return 500, J, {"message": "Could not find the volume"}
            if method == "GET":
                return 200, J, v
            action = p.rsplit("/", 1)[-1]
            if action == "addMappedSdc":
                if v["mappedSdcInfo"] and body["allowMultipleMappings"] != "TRUE":
                    return 500, J, {"message": "volume already mapped"}
                v["mappedSdcInfo"].append({"sdcId": body["sdcId"]})
                if self.sdcs[body["sdcId"]] != "OTHER-GUID":
                    os.makedirs(self.by_id, exist_ok=True)
                    open(self._dev(vid), "w").close()
            elif action == "removeMappedSdc":
                v["mappedSdcInfo"] = [x for x in v["mappedSdcInfo"] if x["sdcId"] != body["sdcId"]]
                if os.path.exists(self._dev(vid)):
                    os.unlink(self._dev(vid))
            elif action == "removeVolume":
                if v["mappedSdcInfo"]:
                    return 500, J, {"message": "volume is mapped"}
                del self.volumes[vid]
            return 200, J, {}
