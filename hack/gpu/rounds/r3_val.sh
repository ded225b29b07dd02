set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3x}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/$TAG/smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/$TAG/bench_n1.log 2>&1 &&
if [ -n "$PROF" ]; then
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_vadd -o vadd -- ./amdkube/_native/bin/rocm-vector-add -n 67108864 > gpurun_out/$TAG/prof_vadd.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_burn -o burn -- ./amdkube/_native/bin/gpu-burn > gpurun_out/$TAG/prof_burn.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_hbm -o hbm -- ./amdkube/_native/bin/hbm-probe > gpurun_out/$TAG/prof_hbm.log 2>&1
fi
echo done
