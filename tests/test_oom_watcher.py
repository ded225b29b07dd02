"""pkg/kubelet/oom_watcher.go: one SystemOOM Warning event on the Node per kernel OOM kill."""
import os

from amdkube.kubelet.oom_watcher import SYSTEM_OOM_EVENT, OOMWatcher, read_oom_kills


class Rec:
    def __init__(self):
        self.events = []

    def event(self, obj, typ, reason, msg):
        self.events.append((obj["kind"], obj["metadata"]["name"], typ, reason, msg))


def _vmstat(path, n):
    path.write_text(f"nr_free_pages 100\noom_kill {n}\npgfault 7\n")


def test_system_oom_events_with_victims(tmp_path):
    vm = tmp_path / "vmstat"
    _vmstat(vm, 3)
    r, w = os.pipe()
    rec = Rec()
    ow = OOMWatcher(rec, lambda: {"kind": "Node", "metadata": {"name": "n1"}}, vmstat=str(vm), kmsg=f"/proc/self/fd/{r}")
    assert ow.poll() == 0 and rec.events == []          # kills before start are not reported
    os.write(w, b"6,1234,5678,-;Out of memory: Killed process 4242 (trainer) total-vm:1kB\n")
    _vmstat(vm, 5)
    assert ow.poll() == 2
    assert rec.events[0] == ("Node", "n1", "Warning", SYSTEM_OOM_EVENT,
                             "System OOM encountered, victim process: trainer, pid: 4242")
    assert rec.events[1][4] == "System OOM encountered"
    assert ow.poll() == 0 and len(rec.events) == 2
    os.close(w)
    os.close(r)


def test_missing_counter_is_not_an_error(tmp_path):
    assert read_oom_kills(str(tmp_path / "absent")) is None
    ow = OOMWatcher(Rec(), lambda: {}, vmstat=str(tmp_path / "absent"), kmsg=None)
    assert ow.poll() == 0
    assert isinstance(read_oom_kills(), (int, type(None)))   # the host's own counter
