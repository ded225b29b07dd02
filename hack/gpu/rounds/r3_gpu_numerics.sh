set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r3e}
mkdir -p gpurun_out/$TAG
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/$TAG/list_avail.txt 2>&1 || true
grep -E "TCC_EA0?_RD|TCC_EA0?_WR|TCC_BUBBLE|TCC_REQ|TCC_READ|TCC_WRITE" gpurun_out/$TAG/list_avail.txt | head -80 > gpurun_out/$TAG/tcc_counters.txt || true
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -k "01 or 04 or 9" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_numerics.log 2>&1
echo done
