set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/val
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/val/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/val/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/val/bench_n1.log 2>&1
