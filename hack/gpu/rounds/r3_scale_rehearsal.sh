# N=1 on the real MI355X, then N=1,2,4,8 on fake devices with pods that live 250 ms (the
# measured HSA vector-add pod lifetime): the node's own work per step at every N.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3sr}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-sched-perf --density-nodes 0 > gpurun_out/$TAG/bench_n1_real.log 2>&1 || exit 1
for N in 1 2 4 8; do
  timeout -k 10 300 python -u bench.py --gpus $N --backend fake --image busybox --pod-arg=-c --pod-arg="sleep 0.25" \
    --steps 15 --warmup 3 --no-sched-perf --density-nodes 0 > gpurun_out/$TAG/fake_n$N.log 2>&1 || exit 1
done
echo done
