# Round 4 end-of-session validation: GPU test tier, smoke, N=1 bench, HBM probe rates, and a
# rocprofv3 kernel-trace summary of the GPU workloads (every step bounded, chained with &&).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4f}
mkdir -p $O
B=./amdkube/_native/bin
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/bench_n1.log 2>&1 &&
timeout -k 10 60 $B/hbm-probe --mib 1024 --iters 20 > $O/hbm_1g.json 2>&1 &&
timeout -k 10 60 $B/hbm-probe --mib 4096 --iters 10 > $O/hbm_4g.json 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o hbm -- $B/hbm-probe --mib 1024 --iters 10 > $O/prof_hbm.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o burn -- $B/gpu-burn --ms 1000 > $O/prof_burn.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o vadd -- $B/rocm-vector-add --json -n 67108864 > $O/prof_vadd.log 2>&1 &&
echo done
