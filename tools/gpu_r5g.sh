#!/bin/bash
# BestFit select stall: the C3 batch without its unconstrained evals (no
# concurrent fast-LFC branch) vs the whole batch; per-eval ticks.
export TMPDIR=/tmp
mkdir -p gpurun_out
BF_ONLY=1 timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/sel_bfonly.log 2>&1 || { echo S1_FAILED; exit 1; }
BF_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_bfonly -o run -- python3 tools/probe_select.py > gpurun_out/kt_bfonly.log 2>&1 || { echo K1_FAILED; exit 1; }
echo rc=0
