"""Merge the ContainerSpecs returned by every plugin's InitContainer into one set of
container run options (reference pkg/kubelet/cm/devicemanager/device_run_container_options.go:24-113):
envs, devices (keyed by container path), mounts (keyed by container path) and annotations
are de-duplicated first-wins; conflicts are logged, never fatal."""
from __future__ import annotations

import logging

log = logging.getLogger("amdkube.devicemanager")


def merge_container_specs(specs: list[dict]) -> dict:
    out = {"envs": {}, "devices": [], "mounts": [], "annotations": {}}
    dev_paths, mount_paths = {}, {}
    for spec in specs:
        for k, v in (spec.get("envs") or {}).items():
            if k in out["envs"] and out["envs"][k] != v:
                log.warning("environment variable %s has conflicting values %r/%r; keeping the first", k, out["envs"][k], v)
                continue
            out["envs"].setdefault(k, v)
        for d in spec.get("devices") or []:
            cp = d["container_path"]
            if cp in dev_paths:
                if dev_paths[cp] != d["host_path"]:
                    log.warning("container device path %s has conflicting host paths %s/%s", cp, dev_paths[cp], d["host_path"])
                continue
            dev_paths[cp] = d["host_path"]
            out["devices"].append(dict(d))
        for mnt in spec.get("mounts") or []:
            cp = mnt["container_path"]
            if cp in mount_paths:
                if mount_paths[cp] != mnt["host_path"]:
                    log.warning("container mount %s has conflicting host paths", cp)
                continue
            mount_paths[cp] = mnt["host_path"]
            out["mounts"].append(dict(mnt))
        for k, v in (spec.get("annotations") or {}).items():
            if k in out["annotations"] and out["annotations"][k] != v:
                log.warning("annotation %s has conflicting values", k)
                continue
            out["annotations"].setdefault(k, v)
    return out
