"""kubeadm upgrade plan / apply (cmd/kubeadm/app/cmd/upgrade/{plan,apply,common}.go,
app/phases/upgrade/{policy,staticpods,postupgrade,versiongetter}.go).

* `plan`: reads the stored MasterConfiguration (kube-system/kubeadm-config), the running
  control-plane mirror pods' versions and this kubeadm's own version, and prints what an
  upgrade would change.
* `apply [VERSION]`: enforces the version skew policy (no downgrade without --force, no
  skipping a minor release, never past kubeadm's own version), then for each component backs
  up its static Pod manifest, writes the re-rendered one (new version, and the --config
  changes if given) and waits until the kubelet has replaced the Pod — the mirror pod's
  config hash changes and the Pod runs (and the API server answers /healthz); on timeout the
  backup is restored. Afterwards the configuration is re-uploaded and the bootstrap RBAC and
  addons are re-applied (postupgrade). `--dry-run` prints the manifests instead.
"""
from __future__ import annotations

import asyncio
import json
import os
import re
import shutil
import sys
import time

import yaml

from .. import GIT_VERSION
from . import _client, _wait_healthy, selfhosting, write_yaml
from .phases import (VERSION_ANNOTATION, control_plane_manifests, load_config_file, merge_config, paths, phase_addons,
                     phase_bootstrap_token, phase_upload_config, read_cluster_config)

COMPONENTS = ("kube-apiserver", "kube-controller-manager", "kube-scheduler")
_MIRROR = "kubernetes.io/config.mirror"


def parse_version(v: str) -> tuple[int, int, int, str]:
    mt = re.match(r"^v?(\d+)\.(\d+)\.(\d+)(.*)$", v or "")
    if not mt:
        raise ValueError(f"invalid version {v!r}")
    return int(mt.group(1)), int(mt.group(2)), int(mt.group(3)), mt.group(4)


def _cmp(a: str, b: str) -> int:
    """Compare versions; the pre-release/build suffix orders lexically after the numbers."""
    x, y = parse_version(a), parse_version(b)
    return (x > y) - (x < y)


def enforce_policy(current: str, target: str, kubeadm_version: str = GIT_VERSION) -> tuple[list, list]:
    """policy.go EnforceVersionPolicies → (skippable errors, mandatory errors)."""
    skippable, mandatory = [], []
    c, t, k = parse_version(current), parse_version(target), parse_version(kubeadm_version)
    if t[0] != c[0]:
        mandatory.append(f"the major version of the target ({target}) differs from the cluster's ({current})")
    if t[:2] > (c[0], c[1] + 1):
        mandatory.append(f"specified version to upgrade to {target} is at least one minor release higher than the "
                         f"cluster version {current}; upgrade one minor release at a time")
    if _cmp(target, current) < 0:
        if t[:2] < c[:2]:
            mandatory.append(f"specified version to upgrade to {target} is lower than the minor release of the cluster {current}")
        else:
            skippable.append(f"specified version to upgrade to {target} is lower than the cluster version {current}")
    if _cmp(target, kubeadm_version) > 0:
        if t[:2] > k[:2]:
            mandatory.append(f"specified version to upgrade to {target} is a newer minor release than kubeadm ({kubeadm_version})")
        else:
            skippable.append(f"specified version to upgrade to {target} is higher than the kubeadm version {kubeadm_version}")
    return skippable, mandatory


async def _mirror(c, name: str, node: str):
    return await c.get_or_none("pods", f"{name}-{node}", "kube-system")


async def component_versions(c, node: str) -> dict[str, str]:
    out = {}
    for comp in COMPONENTS:
        p = await _mirror(c, comp, node)
        out[comp] = ((p or {}).get("metadata", {}).get("annotations") or {}).get(VERSION_ANNOTATION, "<unknown>")
    return out


async def plan(a) -> int:
    c = _client(a.kubeconfig)
    try:
        mc = await read_cluster_config(c)
        if mc is None:
            print(f"[upgrade/config] FATAL: the ConfigMap kube-system/kubeadm-config does not exist; run "
                  "`kubeadm config upload` first", file=sys.stderr)
            return 1
        node = mc.get("nodeName")
        vers = await component_versions(c, node)
        target = GIT_VERSION
        print("[upgrade/config] Making sure the configuration is correct: read kube-system/kubeadm-config")
        print(f"[upgrade] Cluster version: {mc.get('kubernetesVersion')}; kubeadm version: {GIT_VERSION}")
        print("\nComponents that will be upgraded after you've upgraded the control plane:")
        print(f"{'COMPONENT':<28}{'CURRENT':<22}AVAILABLE")
        for comp, v in vers.items():
            print(f"{comp:<28}{v:<22}{target}")
        sk, mand = enforce_policy(mc.get("kubernetesVersion") or GIT_VERSION, target)
        if mand:
            print("\n[upgrade/versions] Upgrade to the latest version is not possible: " + "; ".join(mand))
        elif _cmp(target, mc.get("kubernetesVersion") or target) == 0 and all(v == target for v in vers.values()):
            print("\nAwesome, you're up-to-date! Enjoy!")
        else:
            print(f"\nYou can now apply the upgrade by executing the following command:\n\n\tkubeadm upgrade apply {target}\n")
        return 0
    finally:
        await c.close()


async def _wait_replaced(c, comp: str, node: str, old_hash: str | None, timeout: float) -> bool:
    """staticpods.go waitForStaticPodHashChange + the component's health."""
    end = time.time() + timeout
    while time.time() < end:
        try:
            p = await _mirror(c, comp, node)
        except Exception:       # the API server itself is restarting
            p = None
        if p is not None:
            h = (p["metadata"].get("annotations") or {}).get(_MIRROR)
            running = (p.get("status") or {}).get("phase") == "Running"
            if h and h != old_hash and running:
                return True
        await asyncio.sleep(0.5)
    return False


async def apply(a) -> int:
    c = _client(a.kubeconfig)
    try:
        stored = await read_cluster_config(c)
        if stored is None:
            print("[upgrade/config] FATAL: the ConfigMap kube-system/kubeadm-config does not exist", file=sys.stderr)
            return 1
        current = stored.get("kubernetesVersion") or GIT_VERSION
        target = a.version or GIT_VERSION
        try:
            sk, mand = enforce_policy(current, target)
        except ValueError as e:
            print(f"[upgrade/version] FATAL: {e}", file=sys.stderr)
            return 1
        if mand or (sk and not a.force):
            for e in mand + sk:
                print(f"[upgrade/version] FATAL: {e}", file=sys.stderr)
            if sk and not mand:
                print("[upgrade/version] pass --force to ignore the skippable errors", file=sys.stderr)
            return 1
        for e in sk:
            print(f"[upgrade/version] WARNING: {e} (forced)")
        mc = merge_config(stored, load_config_file(a.config)) if a.config else dict(stored)
        mc["kubernetesVersion"] = target
        p = paths(a.base_dir, mc)
        manifests = control_plane_manifests(mc, p)
        if a.dry_run:
            for comp in COMPONENTS:
                print(f"[dryrun] Would write {os.path.join(p['manifests'], comp + '.yaml')}:")
                print(yaml.safe_dump(manifests[comp], sort_keys=False))
            return 0
        if not a.yes and sys.stdin.isatty():
            if input(f"[upgrade/confirm] Are you sure you want to proceed with the upgrade to {target}? [y/N]: ").strip().lower() != "y":
                print("[upgrade] aborted")
                return 1
        node = mc.get("nodeName")
        backup = os.path.join(a.base_dir, "tmp", f"kubeadm-backup-manifests-{time.strftime('%Y%m%d%H%M%S')}")
        os.makedirs(backup, exist_ok=True)
        print(f"[upgrade/staticpods] Writing new Static Pod manifests to {p['manifests']} (backup in {backup})")
        for comp in COMPONENTS:
            path = os.path.join(p["manifests"], f"{comp}.yaml")
            ds = await c.get_or_none("daemonsets.apps", selfhosting.PREFIX + comp, "kube-system")
            if ds is not None and not os.path.exists(path):
                # a self-hosted component: roll its DaemonSet (selfhosted upgrade path) instead of a manifest
                rc = await _upgrade_self_hosted(c, comp, ds, manifests[comp], a.timeout, p)
                if rc:
                    return rc
                continue
            mirror = await _mirror(c, comp, node)
            old_hash = ((mirror or {}).get("metadata", {}).get("annotations") or {}).get(_MIRROR)
            if os.path.exists(path):
                shutil.copy2(path, os.path.join(backup, f"{comp}.yaml"))
                if yaml.safe_load(open(path)) == manifests[comp]:
                    print(f"[upgrade/staticpods] {comp} is unchanged")
                    continue
            write_yaml(path, manifests[comp], 0o644)
            ok = await _wait_replaced(c, comp, node, old_hash, a.timeout)
            if ok and comp == "kube-apiserver":
                ok = await _wait_healthy(c, a.timeout)
            if not ok:
                print(f"[upgrade/staticpods] {comp} did not come back in {a.timeout:.0f}s; rolling back to the backup",
                      file=sys.stderr)
                shutil.copy2(os.path.join(backup, f"{comp}.yaml"), path)
                await _wait_replaced(c, comp, node, None, a.timeout)
                return 1
            print(f"[upgrade/staticpods] Component {comp} upgraded successfully")
        print("[upgrade/postupgrade] Re-uploading the configuration, bootstrap RBAC and addons")
        await phase_upload_config(c, mc)
        for which in ("allow-post-csrs", "allow-auto-approve", "cluster-info"):
            await phase_bootstrap_token(c, mc, p, which)
        await phase_addons(c, mc, p, "kube-proxy")
        await phase_addons(c, mc, p, "kube-dns")
        print(f"\n[upgrade/successful] SUCCESS! Your cluster was upgraded to \"{target}\". Enjoy!")
        return 0
    finally:
        await c.close()


async def _upgrade_self_hosted(c, comp: str, ds: dict, manifest: dict, timeout: float, p: dict) -> int:
    # a plane converted with StoreCertsInSecrets keeps reading its Secrets
    vols = {v.get("name") for v in ds["spec"]["template"]["spec"].get("volumes") or []}
    secrets = (p["pki"], p["kubeconfig_dir"]) if vols & {selfhosting.CERTS_VOLUME, selfhosting.KUBECONFIG_VOLUME} else None
    new = selfhosting.build_daemonset(comp, json.loads(json.dumps(manifest.get("spec") or {})), secrets)

    def key(spec):       # what a manifest decides; the stored template also carries API defaults
        return [(c.get("name"), c.get("image"), c.get("command"), c.get("args"), c.get("env")) for c in spec.get("containers") or []]
    if key(ds["spec"]["template"]["spec"]) == key(new["spec"]["template"]["spec"]):
        print(f"[upgrade/selfhosted] {comp} is unchanged")
        return 0
    ds["spec"]["template"] = new["spec"]["template"]
    await selfhosting.create_or_update_daemonset(c, dict(ds, apiVersion="apps/v1", kind="DaemonSet"))
    want = new["spec"]["template"]["spec"]["containers"][0].get("args")

    async def rolled():
        pods, _ = await c.list("pods", "kube-system", label_selector=f"k8s-app={selfhosting.PREFIX}{comp}")
        return bool(pods) and all(p["spec"]["containers"][0].get("args") == want
                                  and (p.get("status") or {}).get("phase") == "Running" for p in pods)
    if not await selfhosting._poll(rolled, timeout) or not await selfhosting._poll(lambda: selfhosting.api_healthy(c), timeout):
        print(f"[upgrade/selfhosted] {comp} did not roll out in {timeout:.0f}s", file=sys.stderr)
        return 1
    print(f"[upgrade/selfhosted] Component {comp} upgraded successfully (DaemonSet {selfhosting.PREFIX}{comp})")
    return 0


def add_parser(sub):
    up = sub.add_parser("upgrade", help="upgrade the control plane")
    us = up.add_subparsers(dest="upgrade_op", required=True)
    pl = us.add_parser("plan")
    pl.add_argument("--kubeconfig", default="/etc/kubernetes/admin.conf")
    ap = us.add_parser("apply")
    ap.add_argument("version", nargs="?", default=None)
    ap.add_argument("--kubeconfig", default="/etc/kubernetes/admin.conf")
    ap.add_argument("--base-dir", default="/etc/kubernetes")
    ap.add_argument("--config", default=None, help="a MasterConfiguration whose fields replace the stored ones")
    ap.add_argument("-y", "--yes", action="store_true")
    ap.add_argument("-f", "--force", action="store_true")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--timeout", type=float, default=120.0)


def run(a) -> int:
    return asyncio.run(plan(a) if a.upgrade_op == "plan" else apply(a))
