#!/bin/bash
# Kernel-trace profile of the C3 bench (no CPU leg): per-kernel stats into gpurun_out/prof.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-extras > gpurun_out/prof_bench.json 2> gpurun_out/prof.log || { echo PROF_FAILED; tail -20 gpurun_out/prof.log; exit 1; }
f=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -30
echo rc=0
