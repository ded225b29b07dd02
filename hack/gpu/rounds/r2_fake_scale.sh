set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2i
for g in 1 2 4 8; do
  timeout -k 10 200 python -u bench.py --gpus $g --steps 10 --warmup 2 --backend fake --no-sched-perf --density-nodes 0 --image busybox --pod-arg=-c --pod-arg=true > gpurun_out/r2i/fake_n$g.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-sched-perf --density-nodes 0 > gpurun_out/r2i/bench_n1.log 2>&1
echo done
