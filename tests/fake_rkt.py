#!/usr/bin/env python3
"""A scripted `rkt` for the rktshim tests: the subset of the rkt 1.x command line the shim uses
(version, fetch, image list/rm, app sandbox/add/start/stop/rm/status/list, status, stop, rm,
enter), with pods and apps as host processes and state under $FAKE_RKT_DIR. Apps write their
output to <kubernetes-log-dir>/<kubernetes-log-path> as the shim asks. No rkt exists offline, so
this stands in for it; it is not a model of rkt's stage1 isolation."""
import hashlib
import json
import os
import signal
import subprocess
import sys
import time
import uuid

ROOT = os.environ.get("FAKE_RKT_DIR", "/tmp/fake-rkt")
IMAGES = {"busybox": ["/bin/sh"], "alpine": ["/bin/sh"], "rocm/vector-add": ["/bin/true"]}


def die(msg, rc=254):
    print(msg, file=sys.stderr)
    sys.exit(rc)


def load(path, default=None):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return default


def save(path, obj):
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


def opts(argv):
    """--k=v flags (repeatable ones collected in lists) and positionals; '--' ends flags."""
    flags, pos, rest = {}, [], []
    for i, a in enumerate(argv):
        if a == "--":
            rest = argv[i + 1:]
            break
        if a.startswith("--"):
            k, _, v = a[2:].partition("=")
            flags.setdefault(k, []).append(v)
        else:
            pos.append(a)
    return flags, pos, rest


def pod_dir(u):
    d = os.path.join(ROOT, "pods", u)
    if not os.path.isdir(d):
        die(f"pod {u} not found")
    return d


def norm(name):
    for p in ("docker://", "docker.io/library/", "docker.io/"):
        if name.startswith(p):
            name = name[len(p):]
    return name if ":" in name.rsplit("/", 1)[-1] else name + ":latest"


def app_status(d, name):
    a = load(os.path.join(d, "apps", name + ".json"))
    if a is None:
        die(f"app {name} not found")
    st = load(os.path.join(d, "apps", name + ".status.json"), {})
    out = {"name": name, "state": st.get("state", "created"), "created_at": a["created_at"],
           "image_id": a["image"], "mounts": a.get("volumes", [])}
    for k in ("started_at", "finished_at", "exit_code", "pid"):
        if k in st:
            out[k] = st[k]
    return out


def cmd_fetch(argv):
    _, pos, _ = opts(argv)
    name = norm(pos[0])
    base = name.rsplit(":", 1)[0]
    if base not in IMAGES:
        die(f"fetch: unable to fetch image from docker://{base}: not found")
    imgs = load(os.path.join(ROOT, "images.json"), [])
    iid = "sha512-" + hashlib.sha512(name.encode()).hexdigest()[:32]
    if not any(i["id"] == iid for i in imgs):
        imgs.append({"id": iid, "name": "registry-1.docker.io/library/" + name if "/" not in base else name,
                     "import_time": time.time_ns(), "size": 1 << 20, "exec": IMAGES[base]})
        save(os.path.join(ROOT, "images.json"), imgs)
    print(iid)


def cmd_image(argv):
    imgs = load(os.path.join(ROOT, "images.json"), [])
    if argv[0] == "list":
        print(json.dumps([{k: v for k, v in i.items() if k != "exec"} for i in imgs]))
    elif argv[0] == "rm":
        save(os.path.join(ROOT, "images.json"), [i for i in imgs if i["id"] not in argv[1:]])


def cmd_sandbox(argv):
    flags, _, _ = opts(argv)
    u = str(uuid.uuid4())
    d = os.path.join(ROOT, "pods", u)
    os.makedirs(os.path.join(d, "apps"))
    ann = dict(x.split("=", 1) for x in flags.get("annotation", []))
    save(os.path.join(d, "pod.json"), {"uuid": u, "state": "running", "pid": os.getpid(), "created_at": time.time_ns(),
                                       "annotations": ann, "hostname": flags.get("hostname", [""])[0],
                                       "net": flags.get("net", ["default"])[0]})
    with open(flags["uuid-file-save"][0], "w") as f:
        f.write(u)

    def stop(*_):
        for a in os.listdir(os.path.join(d, "apps")):
            if a.endswith(".status.json"):
                st = load(os.path.join(d, "apps", a), {})
                if st.get("state") == "running" and st.get("pid"):
                    try:
                        os.killpg(st["pid"], signal.SIGKILL)
                    except OSError:
                        pass
        pod = load(os.path.join(d, "pod.json"))
        pod["state"] = "exited"
        save(os.path.join(d, "pod.json"), pod)
        sys.exit(0)
    signal.signal(signal.SIGTERM, stop)
    while True:
        time.sleep(3600)


def cmd_app(argv):
    sub, rest = argv[0], argv[1:]
    flags, pos, tail = opts(rest)
    d = pod_dir(pos[0])
    if sub == "add":
        imgs = {i["id"]: i for i in load(os.path.join(ROOT, "images.json"), [])}
        img = imgs.get(pos[1]) or die(f"image {pos[1]} not found")
        name = flags["name"][0]
        if os.path.exists(os.path.join(d, "apps", name + ".json")):
            die(f"app {name} already exists")
        exe = flags.get("exec", [None])[0]
        argv_ = ([exe] + tail) if exe else (img["exec"] + tail)
        vols = []
        for v in flags.get("mnt-volume", []):
            vols.append(dict(kv.split("=", 1) for kv in v.split(",")))
        save(os.path.join(d, "apps", name + ".json"), {
            "name": name, "image": pos[1], "argv": argv_, "created_at": time.time_ns(),
            "env": dict(x.split("=", 1) for x in flags.get("environment", [])),
            "annotations": dict(x.split("=", 1) for x in flags.get("annotation", [])),
            "workdir": flags.get("working-dir", [""])[0], "volumes": vols})
    elif sub == "start":
        name = flags["app"][0]
        app_status(d, name)
        subprocess.Popen([sys.executable, os.path.abspath(__file__), "_run", pos[0], name], start_new_session=True,
                         stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        for _ in range(500):
            if app_status(d, name)["state"] != "created":
                return
            time.sleep(0.01)
        die("app did not start")
    elif sub == "stop":
        name = flags["app"][0]
        st = app_status(d, name)
        if st["state"] == "running":
            try:
                os.killpg(st["pid"], signal.SIGTERM)
            except OSError:
                pass
            for _ in range(500):
                if app_status(d, name)["state"] == "exited":
                    return
                time.sleep(0.01)
            os.killpg(st["pid"], signal.SIGKILL)
    elif sub == "rm":
        name = flags["app"][0]
        for suffix in (".json", ".status.json"):
            try:
                os.unlink(os.path.join(d, "apps", name + suffix))
            except OSError:
                pass
    elif sub == "status":
        print(json.dumps(app_status(d, flags["app"][0])))
    elif sub == "list":
        print(json.dumps([app_status(d, a[:-5]) for a in sorted(os.listdir(os.path.join(d, "apps")))
                          if a.endswith(".json") and not a.endswith(".status.json")]))
    else:
        die(f"unknown app subcommand {sub}")


def run_app(u, name):
    """The per-app supervisor (stage1's job): run the app, record pid / start / exit."""
    d = pod_dir(u)
    a = load(os.path.join(d, "apps", name + ".json"))
    pod = load(os.path.join(d, "pod.json"))
    logp = os.path.join(pod["annotations"].get("coreos.com/rkt/experiment/kubernetes-log-dir", d),
                        a["annotations"].get("coreos.com/rkt/experiment/kubernetes-log-path", name + ".log"))
    os.makedirs(os.path.dirname(logp), exist_ok=True)
    env = {"PATH": "/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin", "HOME": "/root", **a["env"]}
    for v in a["volumes"]:      # apps see their volumes under the pod's root, as symlinks
        env.setdefault("RKT_VOLUME_" + v["name"].upper().replace("-", "_"), v["source"])
    log = open(logp, "ab")
    p = subprocess.Popen(a["argv"], stdout=log, stderr=log, stdin=subprocess.DEVNULL, env=env,
                         cwd=a["workdir"] or None, start_new_session=True)
    sp = os.path.join(d, "apps", name + ".status.json")
    save(sp, {"state": "running", "pid": p.pid, "started_at": time.time_ns()})
    rc = p.wait()
    st = load(sp, {})
    st.update(state="exited", exit_code=rc if rc >= 0 else 128 - rc, finished_at=time.time_ns())
    save(sp, st)


def main():
    os.makedirs(os.path.join(ROOT, "pods"), exist_ok=True)
    argv = [a for a in sys.argv[1:] if not a.startswith("--format=") and not a.startswith("--insecure-options")
            and a != "--full" and a != "--debug"]
    if not argv:
        die("usage: rkt COMMAND")
    cmd, rest = argv[0], argv[1:]
    if cmd == "version":
        print("rkt Version: 1.30.0\nappc Version: 0.8.11\nGo Version: go1.9\nFeatures: -TPM +SDJOURNAL")
    elif cmd == "fetch":
        cmd_fetch(rest)
    elif cmd == "image":
        cmd_image(rest)
    elif cmd == "app" and rest and rest[0] == "sandbox":
        cmd_sandbox(rest[1:])
    elif cmd == "app":
        cmd_app(rest)
    elif cmd == "_run":
        run_app(rest[0], rest[1])
    elif cmd == "status":
        _, pos, _ = opts(rest)
        d = pod_dir(pos[0])
        pod = load(os.path.join(d, "pod.json"))
        apps = sorted(a[:-5] for a in os.listdir(os.path.join(d, "apps")) if a.endswith(".json") and not a.endswith(".status.json"))
        print(json.dumps({"name": pod["uuid"], "state": pod["state"], "pid": pod["pid"], "created_at": pod["created_at"],
                          "app_names": apps, "networks": [] if pod["net"] == "host" else [{"netName": "default", "ip": "10.1.0.2"}]}))
    elif cmd == "stop":
        _, pos, _ = opts(rest)
        pod = load(os.path.join(pod_dir(pos[0]), "pod.json"))
        if pod["state"] == "running":
            try:
                os.kill(pod["pid"], signal.SIGTERM)
            except OSError:
                pass
    elif cmd == "rm":
        _, pos, _ = opts(rest)
        import shutil
        shutil.rmtree(pod_dir(pos[0]), ignore_errors=True)
    elif cmd == "enter":
        flags, pos, _ = opts(rest[:2])
        d = pod_dir(pos[0])
        a = load(os.path.join(d, "apps", flags["app"][0] + ".json"))
        env = {"PATH": "/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin", **a["env"]}
        os.execvpe(rest[2], rest[2:], env)
    else:
        die(f"unknown command {cmd}")


if __name__ == "__main__":
    main()
