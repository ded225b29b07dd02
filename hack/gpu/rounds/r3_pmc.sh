# PMC passes that settle how FETCH_SIZE weighs gfx950's read requests:
# the raw TCC EA request counters by size next to FETCH_SIZE / WRITE_SIZE, on the HBM probe
# and the 64 M-element vector add. One counter group per run (rocprofv3 does not multiplex).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r3pmc}
mkdir -p gpurun_out/$TAG
B=./amdkube/_native/bin
run() {   # name, counters, argv...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/$TAG/$name -o $name -- "$@" > gpurun_out/$TAG/$name.log 2>&1
}
for w in hbm vadd; do
  if [ $w = hbm ]; then W="$B/hbm-probe --mib 1024 --iters 2"; else W="$B/rocm-vector-add -n 67108864"; fi
  run ${w}_rdreq "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum" $W &&
  run ${w}_fetch "FETCH_SIZE" $W &&
  run ${w}_write "WRITE_SIZE" $W &&
  run ${w}_wrreq "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" $W || exit 1
done
echo done
