#!/bin/bash
# Per-eval select profile (profiling build) then the round's evidence
# (tools/gpu_final.sh: bench, kernel trace, PMC, probes).  Chained.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/probe_select.log 2>&1 || { echo SELECT_PROBE_FAILED; exit 1; }
bash tools/gpu_final.sh
