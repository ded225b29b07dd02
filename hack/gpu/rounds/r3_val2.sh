set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3y}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/$TAG/smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench_n1.log 2>&1 &&
timeout -k 10 150 python -u hack/gpu/experiments/concurrent_procs.py > gpurun_out/$TAG/concurrent_procs.jsonl 2>&1 &&
for E in 0 1000; do
  for N in 100 1000; do
    timeout -k 10 300 python -u -m amdkube.benchmark.schedperf --nodes $N --pods 1000 --existing $E --gpu-pods mixed > gpurun_out/$TAG/schedperf_n${N}_e${E}.json 2> gpurun_out/$TAG/schedperf_n${N}_e${E}.err || exit 1
  done
done
echo done
