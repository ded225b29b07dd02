"""Diagnostic: does amd-smi's process list report PIDs in our namespace?"""
import os, subprocess, sys, time, json
sys.path.insert(0, os.getcwd())
from amdkube.smi.backend import open_backend
b = open_backend("amdsmi")
p = subprocess.Popen(["./amdkube/_native/bin/gpu-burn", "--ms", "4000"], stdout=subprocess.DEVNULL)
time.sleep(2.0)
out = {"child_pid": p.pid, "self_pid": os.getpid(), "uid": os.getuid(),
       "pidns": os.readlink("/proc/self/ns/pid"), "init_pidns": None}
try:
    out["init_pidns"] = os.readlink("/proc/1/ns/pid")
except OSError as e:
    out["init_pidns"] = str(e)
try:
    out["kfd_proc"] = sorted(os.listdir("/sys/class/kfd/kfd/proc"))[:20]
except OSError as e:
    out["kfd_proc"] = str(e)
for g in b.gpus()[:2]:
    out[f"gpu{g['index']}"] = b.processes(g["index"])
try:
    out["status_nspid"] = [l for l in open(f"/proc/{p.pid}/status") if l.startswith("NSpid")]
except OSError as e:
    out["status_nspid"] = str(e)
p.wait()
print(json.dumps(out, default=str))
