#!/bin/bash
# The GPU evidence runner (run from the repository root on an MI355X box, e.g. through gpurun):
#   bash hack/gpu/run.sh tier      GPU test tier, smoke(), 1-GPU bench.py     -> gpurun_out/{pytest_gpu,smoke,bench_n1}.log
#   bash hack/gpu/run.sh profile   rocprofv3 kernel traces + summaries of the native GPU tools,
#                                  then the tier, then one counter pass        -> gpurun_out/prof_*, sum_*, pmc_*
# Every GPU step runs under its own timeout; the first failure ends the run.
set -e
case "${1:-tier}" in
  tier) bash "$(dirname "$0")/tier.sh" ;;
  profile) bash "$(dirname "$0")/profile.sh" ;;
  *) echo "usage: $0 tier|profile" >&2; exit 2 ;;
esac
