# Kernel-trace summaries (rocprofv3 --kernel-trace --stats, no PMC) of the GPU workloads at the
# end of round 3: the pod workload on bare ROCr, its HIP twin, the HBM probe, the MFMA burn.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r3final}
mkdir -p gpurun_out/$TAG
B=./amdkube/_native/bin
prof() {   # name, argv...
  local name=$1; shift
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/$name -o $name -- "$@" \
    > gpurun_out/$TAG/$name.log 2>&1
}
prof hsa_vadd $B/hsa-vector-add -n 67108864 &&
prof hip_vadd $B/rocm-vector-add -n 67108864 &&
prof hbm $B/hbm-probe --mib 1024 --iters 4 &&
prof burn $B/gpu-burn --ms 500 &&
for f in $(find gpurun_out/$TAG -name "*kernel_stats.csv" | sort); do echo "## $f"; cat "$f"; done > gpurun_out/$TAG/kernel_stats_all.txt
echo done
