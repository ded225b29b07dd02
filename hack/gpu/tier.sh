#!/bin/bash
# GPU evidence pass: GPU test tier, 1-GPU bench (GPU pods + scheduler_perf + density), smoke.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python bench.py --steps 20 --warmup 2 > gpurun_out/bench_n1.log 2>&1
echo done
