"""Stateful property tests of the GPU allocation invariants (Hypothesis drives the
allocator and the scheduler cache through random interleavings). Whatever the order of pod
schedules / binds / deletions, node updates and device health flips:

  * no device is ever assigned to two live pods of a node (the reference's defect #1),
  * an unhealthy device is never handed out (defect #6),
  * a node's available set is exactly its healthy devices minus the assigned ones,
  * a pod that asks for k GPUs gets k distinct devices of that node,
  * the native topology selector returns distinct candidates of the requested size.
"""
import asyncio
import copy

from hypothesis import HealthCheck, given, settings, strategies as st
from hypothesis.stateful import RuleBasedStateMachine, initialize, invariant, precondition, rule

from amdkube.ops import topology as topo
from amdkube.scheduler.cache import SchedulerCache
from amdkube.scheduler.generic import FitError, GenericScheduler
from amdkube.scheduler.predicates import DEFAULT_PREDICATES
from amdkube.scheduler.priorities import DEFAULT_PRIORITIES
from tests.test_scheduler import node, pod

R = "amd.com/gpu"


class AllocatorMachine(RuleBasedStateMachine):
    @initialize()
    def setup(self):
        self.nodes = {n: node(n, gpus=8) for n in ("n0", "n1")}
        self.cache = SchedulerCache()
        for n in self.nodes.values():
            self.cache.add_node(copy.deepcopy(n))
        self.sched = GenericScheduler(self.cache, list(DEFAULT_PREDICATES), dict(DEFAULT_PRIORITIES))
        self.pods: dict[str, dict] = {}
        self.seq = 0

    def _healthy(self, n):
        return {d for d, x in self.nodes[n]["status"]["extendedResources"][R]["resources"].items() if x["health"] == "Healthy"}

    @rule(k=st.sampled_from([1, 1, 2, 4, 8]), bind=st.booleans())
    def schedule(self, k, bind):
        self.seq += 1
        name = f"p{self.seq}"
        try:
            host, binding = asyncio.run(self.sched.schedule(pod(name, k)))
        except FitError:
            free = {n: len(self.cache.nodes[n].available_devices(R)) for n in self.nodes}
            assert all(v < k for v in free.values()), (k, free)
            return
        ids = binding["gpus"]["resources"]
        assert len(ids) == k and len(set(ids)) == k
        assert set(ids) <= self._healthy(host)
        p = pod(name, k, node_name=host, assigned={"gpus": ids})
        if bind:
            self.cache.add_pod(p)          # the informer saw the bound pod
        else:
            self.cache.assume_pod(p)       # assumed, binding in flight
        self.pods[name] = p

    @precondition(lambda self: self.pods)
    @rule(data=st.data())
    def delete(self, data):
        name = data.draw(st.sampled_from(sorted(self.pods)))
        p = self.pods.pop(name)
        if self.cache.is_assumed(p) and data.draw(st.booleans()):
            self.cache.forget_pod(p)       # binding failed
        else:
            self.cache.remove_pod(p)

    @rule(n=st.sampled_from(["n0", "n1"]), i=st.integers(0, 7), healthy=st.booleans())
    def flip_health(self, n, i, healthy):
        devs = self.nodes[n]["status"]["extendedResources"][R]["resources"]
        did = sorted(devs)[i]
        devs[did]["health"] = "Healthy" if healthy else "Unhealthy"
        self.cache.add_node(copy.deepcopy(self.nodes[n]))      # node update event

    @invariant()
    def no_double_assignment_and_exact_availability(self):
        for n in self.nodes:
            live = [p for p in self.pods.values() if p["spec"]["nodeName"] == n]
            assigned = [d for p in live for d in p["spec"]["extendedResources"][0]["assigned"]]
            assert len(assigned) == len(set(assigned)), "device assigned twice"
            avail = set(self.cache.nodes[n].available_devices(R))
            assert avail == self._healthy(n) - set(assigned)


TestAllocator = AllocatorMachine.TestCase
TestAllocator.settings = settings(max_examples=60, stateful_step_count=30, deadline=None,
                                  suppress_health_check=[HealthCheck.too_slow])


@settings(max_examples=200, deadline=None)
@given(st.data())
def test_native_topology_select_returns_distinct_candidates(data):
    n_gpus = 8
    link = [[0 if i == j else (15 if (i // 4) == (j // 4) else 30) for j in range(n_gpus)] for i in range(n_gpus)]
    numa = [i // 4 for i in range(n_gpus)]
    parent = [i // 2 for i in range(n_gpus)]
    free = sorted(data.draw(st.sets(st.integers(0, n_gpus - 1), min_size=1)))
    cand = sorted(data.draw(st.sets(st.sampled_from(free), min_size=1)))
    k = data.draw(st.integers(1, len(cand)))
    sel, cost = topo.select(cand, k, link, numa, free, parent)
    assert len(sel) == k and len(set(sel)) == k and set(sel) <= set(cand)
