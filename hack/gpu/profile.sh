#!/bin/bash
# One GPU evidence pass: rocprofv3 kernel traces + summaries, pytest -m gpu, bench, counters last.
set -e
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for spec in "hbm:hbm-probe --mib 4096 --iters 20" "burn:gpu-burn --ms 2000" "vadd:rocm-vector-add --json -n 67108864"; do
  n=${spec%%:*}; cmd=${spec#*:}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$n -o $n -- $R/amdkube/_native/bin/$cmd > $R/gpurun_out/$n.json
  timeout -k 10 60 /opt/rocm/bin/rocpd2summary -i $(ls $R/gpurun_out/prof_$n/*.db) -f md -d $R/gpurun_out/sum_$n -o $n > /dev/null 2>&1 || true
done
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 2 > gpurun_out/bench_n1.log 2>&1
cd /tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_avail.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_burn -o burn --output-format csv -- $R/amdkube/_native/bin/gpu-burn --ms 200 > $R/gpurun_out/burn_pmc.json 2> $R/gpurun_out/burn_pmc.err
echo done
