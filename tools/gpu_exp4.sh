#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/exp_knobs.sh KTAS_BENCH_HOST_VALUES 0 1 0 1 || exit 1
timeout -k 10 120 python tools/probe_trace.py C3 > gpurun_out/trace_pin1.log 2>&1 && tail -1 gpurun_out/trace_pin1.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e4 -o run -- python3 bench.py --no-cpu --no-extras --steps 20 --warmup 5 > gpurun_out/prof_e4_bench.json 2> gpurun_out/prof_e4.log || { echo PROF_FAILED; exit 1; }
echo rc=0
