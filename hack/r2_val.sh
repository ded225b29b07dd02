set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r2/smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2/bench_n1.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_bench -o run -- python3 bench.py --steps 5 --warmup 1 --no-sched-perf --density-nodes 0 > gpurun_out/r2/bench_prof.log 2>&1
echo done
