# Round 4: HBM write-front validation (GPU tests of the probe kernels, probe rates at 1 and 4 GiB,
# a kernel-trace profile of the probe, and the vector-add front sweep).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-hb6}
mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu.py -k "test_95 or test_92 or test_94" -x -q --timeout 100 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 60 ./amdkube/_native/bin/hbm-probe --mib 1024 --iters 20 > $O/hbm_1g.json 2>&1 &&
timeout -k 10 60 ./amdkube/_native/bin/hbm-probe --mib 4096 --iters 10 > $O/hbm_4g.json 2>&1 &&
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $O/prof -o hbm -- ./amdkube/_native/bin/hbm-probe --mib 1024 --iters 10 > $O/prof.log 2>&1 &&
timeout -k 10 60 hack/gpu/experiments/vadd_front6 > $O/vadd_front6.jsonl 2>&1 &&
echo done
