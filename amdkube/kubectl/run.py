"""kubectl run and its generators.

Reference: pkg/kubectl/cmd/run.go RunRun (:147-410) and pkg/kubectl/run.go —
  * validation: NAME, --image (a docker reference), -t needs -i, -i needs --replicas=1,
    --expose needs --port, --restart other than Always needs --replicas=1, --rm only when
    attached, --dry-run never when attached, --image-pull-policy Always|IfNotPresent|Never;
  * getRestartPolicy (:487-505): empty means OnFailure when interactive, else Always;
  * the generator (:218-263): --schedule → cronjob/v1beta1 (cronjob/v2alpha1 when the server
    lacks batch/v1beta1 cronjobs); Always → deployment/v1beta1 (run/v1 when extensions
    deployments are not served); OnFailure → job/v1 (run-pod/v1 without batch/v1 jobs);
    Never → run-pod/v1; --generator picks one by name;
  * the generators (run.go): labels `run=<name>` unless --labels; the container is named after
    the workload; trailing arguments are args, or the command with --command; --env KEY=VALUE
    (parseEnvs); --port / --hostport (hostport needs port); --requests / --limits
    (`cpu=100m,memory=256Mi`); --serviceaccount; run-pod/v1 sets IfNotPresent, ClusterFirst
    and StdinOnce = stdin && !--leave-stdin-open; Job/CronJob default to restartPolicy Never;
    CronJob uses concurrencyPolicy Allow; ValidateParams: "Parameter: X is required";
  * --overrides: a JSON patch merged into the generated object (cmdutil.Merge, strategic);
  * --expose: a service/v2 Service selecting the workload's labels on --port;
  * --attach / -i: wait for the pod, stream its output (amdkube's attach is output-only), with
    --restart=Never return the container's exit code, --rm deletes what was created.
amdkube: --gpus N adds an `amd.com/gpu: N` limit to the container.
"""
from __future__ import annotations

import asyncio
import json
import re
import sys

from ..api import meta as m
from ..api.quantity import Quantity

# docker/distribution reference.ReferenceRegexp
_ALNUM = r"[a-z0-9]+"
_SEP = r"(?:[._]|__|[-]*)"
_COMPONENT = _ALNUM + r"(?:" + _SEP + _ALNUM + r")*"
_DOMAIN_COMP = r"(?:[a-zA-Z0-9]|[a-zA-Z0-9][a-zA-Z0-9-]*[a-zA-Z0-9])"
_DOMAIN = _DOMAIN_COMP + r"(?:\." + _DOMAIN_COMP + r")*(?::[0-9]+)?"
_NAME = r"(?:" + _DOMAIN + r"/)?" + _COMPONENT + r"(?:/" + _COMPONENT + r")*"
REFERENCE_RE = re.compile(r"^" + _NAME + r"(?::[\w][\w.-]{0,127})?(?:@[A-Za-z][A-Za-z0-9]*(?:[-_+.][A-Za-z][A-Za-z0-9]*)*"
                          r":[0-9a-fA-F]{32,})?$")
ENV_NAME_RE = re.compile(r"^[-._a-zA-Z][-._a-zA-Z0-9]*$")

GENERATORS = ("run/v1", "run-pod/v1", "deployment/v1beta1", "deployment/apps.v1beta1", "job/v1", "cronjob/v1beta1",
              "cronjob/v2alpha1")
PARAMS = {
    "run/v1": ("labels", "default-name", "name!", "replicas!", "image!", "image-pull-policy", "port", "hostport", "stdin",
               "tty", "command", "args", "env", "requests", "limits", "serviceaccount"),
    "run-pod/v1": ("labels", "default-name", "name!", "image!", "image-pull-policy", "port", "hostport", "stdin",
                   "leave-stdin-open", "tty", "restart", "command", "args", "env", "requests", "limits", "serviceaccount"),
    "deployment/v1beta1": ("labels", "default-name", "name!", "replicas!", "image!", "image-pull-policy", "port", "hostport",
                           "stdin", "tty", "command", "args", "env", "requests", "limits", "serviceaccount"),
    "job/v1": ("labels", "default-name", "name!", "image!", "image-pull-policy", "port", "hostport", "stdin",
               "leave-stdin-open", "tty", "command", "args", "env", "requests", "limits", "restart", "serviceaccount"),
    "cronjob/v1beta1": ("labels", "default-name", "name!", "image!", "image-pull-policy", "port", "hostport", "stdin",
                        "leave-stdin-open", "tty", "command", "args", "env", "requests", "limits", "restart", "schedule!",
                        "serviceaccount"),
}
PARAMS["deployment/apps.v1beta1"] = PARAMS["deployment/v1beta1"]
PARAMS["cronjob/v2alpha1"] = PARAMS["cronjob/v1beta1"]


class GenerateError(ValueError):
    pass


def get_bool(params: dict, key: str, default: bool = False) -> bool:
    """GetBool → strconv.ParseBool."""
    if key not in params:
        return default
    v = params[key]
    if v in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if v in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    raise GenerateError(f'strconv.ParseBool: parsing "{v}": invalid syntax')


def parse_labels_spec(spec: str) -> dict:
    """kubectl.ParseLabels: `a=b,c=d`."""
    if not spec:
        raise GenerateError("no label spec passed")
    out = {}
    for part in spec.split(","):
        kv = part.split("=")
        if len(kv) != 2:
            raise GenerateError(f"unexpected label spec: {part}")
        if not kv[0]:
            raise GenerateError("unexpected empty label key")
        out[kv[0]] = kv[1]
    return out


def parse_envs(envs) -> list[dict]:
    out = []
    for e in envs:
        pos = e.find("=")
        if pos <= 0 or not ENV_NAME_RE.match(e[:pos]):
            raise GenerateError(f"invalid env: {e}")
        out.append({"name": e[:pos], "value": e[pos + 1:]})
    return out


def resource_list(spec: str) -> dict | None:
    """populateResourceListV1: `cpu=100m,memory=256Mi`; empty → nil."""
    if not spec:
        return None
    out = {}
    for stmt in spec.split(","):
        parts = stmt.split("=")
        if len(parts) != 2:
            raise GenerateError(f"Invalid argument syntax {stmt}, expected <resource>=<value>")
        try:
            Quantity(parts[1])
        except Exception:
            raise GenerateError("quantities must match the regular expression '^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$'") from None
        out[parts[0]] = parts[1]
    return out


def validate_params(generator: str, params: dict):
    errs = [f"Parameter: {p[:-1]} is required" for p in PARAMS[generator]
            if p.endswith("!") and not params.get(p[:-1])]
    if errs:
        raise GenerateError(errs[0] if len(errs) == 1 else "[" + ", ".join(errs) + "]")


def _name(params):
    name = params.get("name") or params.get("default-name")
    if not name:
        raise GenerateError("'name' is a required parameter.")
    return name


def _labels(params, name):
    return parse_labels_spec(params["labels"]) if params.get("labels") else {"run": name}


def _pod_spec(params, name, basic_pod=False) -> dict:
    """makePodSpec + updatePodContainers + updatePodPorts."""
    stdin, tty = get_bool(params, "stdin"), get_bool(params, "tty")
    res = {}
    lim, req = resource_list(params.get("limits", "")), resource_list(params.get("requests", ""))
    if lim:
        res["limits"] = lim
    if req:
        res["requests"] = req
    c = {"name": name, "image": params.get("image", "")}
    if basic_pod:
        c["imagePullPolicy"] = "IfNotPresent"
    if stdin:
        c["stdin"] = True
    if tty:
        c["tty"] = True
    if res:
        c["resources"] = res
    spec = {"containers": [c]}
    if params.get("serviceaccount"):
        spec["serviceAccountName"] = params["serviceaccount"]
    args = params.get("args") or []
    if args:
        c["command" if get_bool(params, "command") else "args"] = list(args)
    if params.get("env"):
        c["env"] = parse_envs(params["env"])
    if params.get("image-pull-policy"):
        c["imagePullPolicy"] = params["image-pull-policy"]
    port = hostport = -1
    if params.get("port"):
        port = int(params["port"])
    if params.get("hostport"):
        hostport = int(params["hostport"])
        if hostport > 0 and port < 0:
            raise GenerateError("--hostport requires --port to be specified")
    if params.get("port"):
        c["ports"] = [{"containerPort": port}]
        if hostport > 0:
            c["ports"][0]["hostPort"] = hostport
    return spec


def _stdin_once(params, spec):
    c = spec["containers"][0]
    if not get_bool(params, "leave-stdin-open") and c.get("stdin"):
        c["stdinOnce"] = True


def generate(generator: str, params: dict) -> dict:
    """The object a run generator makes from its parameters (strings, `args`/`env` lists)."""
    params = dict(params)
    validate_params(generator, params)
    name = _name(params)
    labels = _labels(params, name)
    if generator == "run-pod/v1":
        spec = _pod_spec(params, name, basic_pod=True)
        _stdin_once(params, spec)
        spec["dnsPolicy"] = "ClusterFirst"
        spec["restartPolicy"] = params.get("restart") or "Always"
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "labels": labels}, "spec": spec}
    spec = _pod_spec(params, name)
    template = {"metadata": {"labels": dict(labels)}, "spec": spec}
    if generator == "run/v1":
        return {"apiVersion": "v1", "kind": "ReplicationController", "metadata": {"name": name, "labels": labels},
                "spec": {"replicas": int(params["replicas"]), "selector": dict(labels), "template": template}}
    if generator in ("deployment/v1beta1", "deployment/apps.v1beta1"):
        api = "extensions/v1beta1" if generator == "deployment/v1beta1" else "apps/v1beta1"
        return {"apiVersion": api, "kind": "Deployment", "metadata": {"name": name, "labels": labels},
                "spec": {"replicas": int(params["replicas"]), "selector": {"matchLabels": dict(labels)}, "template": template}}
    _stdin_once(params, spec)
    spec["restartPolicy"] = params.get("restart") or "Never"
    if generator == "job/v1":
        return {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": name, "labels": labels},
                "spec": {"template": template}}
    api = "batch/v1beta1" if generator == "cronjob/v1beta1" else "batch/v2alpha1"
    return {"apiVersion": api, "kind": "CronJob", "metadata": {"name": name, "labels": labels},
            "spec": {"schedule": params["schedule"], "concurrencyPolicy": "Allow",
                     "jobTemplate": {"spec": {"template": template}}}}


def generate_service(params: dict) -> dict:
    """service/v2 from run's string parameters (generateService :518-566)."""
    name = params.get("name")
    if not name:
        raise GenerateError("name is a required parameter")
    selector = params.get("labels") or f"run={name}"
    port = params.get("port")
    if not port:
        raise GenerateError("'port' is a required parameter.")
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": params.get("default-name") or name},
           "spec": {"selector": parse_labels_spec(selector),
                    "ports": [{"port": int(port), "protocol": "TCP", "targetPort": int(port)}]}}
    if params.get("labels"):
        svc["metadata"]["labels"] = parse_labels_spec(params["labels"])
    return svc


def get_restart_policy(restart: str | None, interactive: bool) -> str:
    if not restart:
        return "OnFailure" if interactive else "Always"
    if restart in ("Always", "OnFailure", "Never"):
        return restart
    raise GenerateError("invalid restart policy: %!s(MISSING)")


def pick_generator(restart: str, schedule: str, served: set[str]) -> str:
    """The default generator (:218-258) from the restart policy and what the server serves
    (`served`: "group/version/resource" strings)."""
    if schedule:
        return "cronjob/v1beta1" if "batch/v1beta1/cronjobs" in served else "cronjob/v2alpha1"
    if restart == "Always":
        return "deployment/v1beta1" if "extensions/v1beta1/deployments" in served else "run/v1"
    if restart == "OnFailure":
        return "job/v1" if "batch/v1/jobs" in served else "run-pod/v1"
    return "run-pod/v1"


def validate(a, name_given: bool):
    """RunRun's checks before anything is generated."""
    if not name_given:
        raise GenerateError("NAME is required for run")
    image = a.image or ""
    if not image:
        raise GenerateError("--image is required")
    if not REFERENCE_RE.match(image):
        raise GenerateError(f'Invalid image name "{image}": invalid reference format')
    interactive, tty = bool(a.stdin), bool(a.tty)
    if tty and not interactive:
        raise GenerateError("-i/--stdin is required for containers with -t/--tty=true")
    replicas = a.replicas if a.replicas is not None else 1
    if interactive and replicas != 1:
        raise GenerateError(f"-i/--stdin requires that replicas is 1, found {replicas}")
    if getattr(a, "expose", False) and not a.port:
        raise GenerateError("--port must be set when exposing a service")
    restart = get_restart_policy(a.restart, interactive)
    if restart != "Always" and replicas != 1:
        raise GenerateError(f"--restart={restart} requires that --replicas=1, found {replicas}")
    attach = a.attach if a.attach is not None else interactive
    if not attach and getattr(a, "rm", False):
        raise GenerateError("--rm should only be used for attached containers")
    if attach and getattr(a, "dry_run", False):
        raise GenerateError("--dry-run can't be used with attached containers options (--attach, --stdin, or --tty)")
    pull = getattr(a, "image_pull_policy", None) or ""
    if pull not in ("", "Always", "IfNotPresent", "Never"):
        raise GenerateError(f"invalid image pull policy: {pull}")
    return restart, replicas, attach


async def _served(c) -> set[str]:
    out = set()
    try:
        groups = await c.request("GET", "/apis")
    except m.StatusError:
        return out
    for g in (groups or {}).get("groups") or []:
        for v in g.get("versions") or []:
            gv = v.get("groupVersion", "")
            try:
                lst = await c.request("GET", f"/apis/{gv}")
            except m.StatusError:
                continue
            out |= {f"{gv}/{r['name']}" for r in (lst or {}).get("resources") or []}
    return out


def _print(obj, fmt):
    if fmt == "json":
        print(json.dumps(obj, indent=4))
    elif fmt == "yaml":
        import yaml
        print(yaml.safe_dump(obj, default_flow_style=False).rstrip())
    elif fmt == "name":
        print(f"{obj['kind'].lower()}/{m.name_of(obj)}")


async def cmd_run(c, a):
    from ..api.strategicpatch import apply as strategic_merge
    from .drain import print_success
    try:
        args = list(a.args)
        restart, replicas, attach = validate(a, bool(args))
        name = args[0]
        generator = getattr(a, "generator", None) or pick_generator(restart, getattr(a, "schedule", "") or "", await _served(c))
        if generator not in GENERATORS:
            raise GenerateError(f'generator "{generator}" not found')
        params = {"name": name, "image": a.image, "replicas": str(replicas), "restart": restart,
                  "labels": a.selector or "", "port": a.port or "", "hostport": str(a.hostport) if a.hostport not in (None, -1) else "",
                  "image-pull-policy": getattr(a, "image_pull_policy", None) or "", "stdin": str(bool(a.stdin)).lower(),
                  "tty": str(bool(a.tty)).lower(), "leave-stdin-open": str(bool(getattr(a, "leave_stdin_open", False))).lower(),
                  "command": str(bool(getattr(a, "command_flag", False))).lower(), "env": list(a.env or []),
                  "requests": a.requests or "", "limits": a.limits or "", "serviceaccount": (getattr(a, "serviceaccount", None) or [""])[-1],
                  "schedule": getattr(a, "schedule", "") or ""}
        params = {k: v for k, v in params.items() if k in {p.rstrip("!") for p in PARAMS[generator]}}
        if a.command:
            params["args"] = list(a.command)
        obj = generate(generator, params)
        if getattr(a, "gpus", 0):
            ctr = (obj["spec"] if obj["kind"] == "Pod" else
                   (obj["spec"]["jobTemplate"]["spec"]["template"]["spec"] if obj["kind"] == "CronJob"
                    else obj["spec"]["template"]["spec"]))["containers"][0]
            ctr.setdefault("resources", {}).setdefault("limits", {})["amd.com/gpu"] = str(a.gpus)
        if getattr(a, "overrides", None):
            obj = strategic_merge(obj, json.loads(a.overrides))
        ns = a.namespace or "default"
        dry = bool(getattr(a, "dry_run", False))
        created = [obj]
        if not dry:
            obj = await c.create(obj, ns)
            created = [obj]
        svc = None
        if getattr(a, "expose", False):
            svc = generate_service({"name": name, "labels": a.selector or "", "port": a.port})
            if getattr(a, "service_overrides", None):
                svc = strategic_merge(svc, json.loads(a.service_overrides))
            if not dry:
                svc = await c.create(svc, ns)
                created.append(svc)
            if a.output or dry:
                _print(svc, a.output or "yaml")
                if a.output == "yaml":
                    print("---")
            else:
                print_success("service", name, "created")
        if attach:
            return await _attach(c, a, ns, obj, restart, created)
        if a.output or dry:
            _print(obj, a.output or "yaml") if a.output else print_success(obj["kind"].lower(), name, "created", dry)
            return 0
        print_success(obj["kind"].lower(), name, "created")
        return 0
    except (GenerateError, ValueError) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1


async def _attach(c, a, ns, obj, restart, created) -> int:
    """Attach (output-only here): wait for the workload's pod, stream its output, and with
    --restart=Never return the container's exit code; --rm deletes what was created."""
    from .logs import first_pod, selector_for_object
    if obj["kind"] == "Pod":
        pod_name = m.name_of(obj)
    else:
        pod, _ = await first_pod(c, ns, selector_for_object(obj) if obj["kind"] != "Job" else
                                 ",".join(f"{k}={v}" for k, v in sorted(((obj["spec"].get("template") or {}).get("metadata")
                                                                          or {}).get("labels", {}).items())),
                                 float(getattr(a, "pod_running_timeout", 60.0) or 60.0))
        pod_name = m.name_of(pod)
    for _ in range(600):
        p = await c.get("pods", pod_name, ns)
        if (p.get("status") or {}).get("phase") in ("Running", "Succeeded", "Failed"):
            break
        await asyncio.sleep(0.1)
    out = sys.stdout.buffer if hasattr(sys.stdout, "buffer") else None
    async for chunk in c.stream_logs(ns, pod_name):
        if out is not None:
            out.write(chunk)
            out.flush()
        else:
            sys.stdout.write(chunk.decode(errors="replace"))
    rc = 0
    if restart == "Never" and not getattr(a, "leave_stdin_open", False):
        for _ in range(600):
            p = await c.get("pods", pod_name, ns)
            phase = (p.get("status") or {}).get("phase")
            if phase in ("Succeeded", "Failed"):
                break
            await asyncio.sleep(0.1)
        if phase == "Failed":
            term = (((p.get("status") or {}).get("containerStatuses") or [{}])[0].get("state") or {}).get("terminated")
            code = int((term or {}).get("exitCode") or 0)
            if not term or code == 0:
                print(f"error: pod {ns}/{pod_name} failed with unknown exit code", file=sys.stderr)
                rc = 1
            else:
                print(f"error: pod {ns}/{pod_name} terminated ({term.get('reason', '')})\n{term.get('message', '')}",
                      file=sys.stderr)
                rc = code
        elif phase != "Succeeded":
            print(f"error: pod {ns}/{pod_name} left in phase {phase}", file=sys.stderr)
            rc = 1
    if getattr(a, "rm", False):
        for o in created:
            ri_plural = {"Pod": "pods", "Service": "services", "Deployment": "deployments", "Job": "jobs",
                         "ReplicationController": "replicationcontrollers", "CronJob": "cronjobs"}[o["kind"]]
            try:
                await c.delete(ri_plural, m.name_of(o), ns, propagation="Background")
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise
    return rc


def add_arguments(sp):
    sp.add_argument("--generator", default=None)
    sp.add_argument("--hostport", type=int, default=-1)
    sp.add_argument("--image-pull-policy", default=None)
    sp.add_argument("--attach", type=lambda s: s.lower() in ("1", "true", "t", "yes"), nargs="?", const=True, default=None)
    sp.add_argument("--rm", action="store_true")
    sp.add_argument("--leave-stdin-open", action="store_true")
    sp.add_argument("--expose", action="store_true")
    sp.add_argument("--overrides", default=None)
    sp.add_argument("--service-overrides", default=None)
    sp.add_argument("--schedule", default="")
    sp.add_argument("--labels", dest="selector", default=argparse_suppress())
    sp.add_argument("--quiet", action="store_true")


def argparse_suppress():
    import argparse
    return argparse.SUPPRESS
