# Round 4: HBM copy layouts (hack/gpu/experiments/copy_sweep3.hip) and 1000-node scheduler_perf on the box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r4b}
mkdir -p gpurun_out/$TAG
timeout -k 10 120 ./hack/gpu/experiments/copy_sweep3 > gpurun_out/$TAG/copy_sweep3.jsonl 2> gpurun_out/$TAG/copy_sweep3.err &&
for e in 0 1000; do
  timeout -k 10 300 python -m amdkube.benchmark.schedperf --nodes 1000 --pods 10000 --existing $e \
    > gpurun_out/$TAG/schedperf_n1000_e${e}_p10000.json 2> gpurun_out/$TAG/schedperf_e${e}.err || exit 1
done &&
timeout -k 10 300 python -m amdkube.benchmark.schedperf --nodes 100 --pods 3000 \
    > gpurun_out/$TAG/schedperf_n100_e0_p3000.json 2> gpurun_out/$TAG/schedperf_n100.err &&
timeout -k 10 300 python hack/proto_vs_json.py > gpurun_out/$TAG/proto_vs_json.json &&
echo done
