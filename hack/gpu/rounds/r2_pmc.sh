set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r2k
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2k/fetch -o fetch -- ./amdkube/_native/bin/hbm-probe --mib 1024 --iters 2 > gpurun_out/r2k/fetch.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2k/write -o write -- ./amdkube/_native/bin/hbm-probe --mib 1024 --iters 2 > gpurun_out/r2k/write.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2k/vadd -o vadd -- ./amdkube/_native/bin/rocm-vector-add -n 67108864 > gpurun_out/r2k/vadd.log 2>&1
echo done
