#!/bin/bash
# Quick C3 bench only (no CPU leg, no extras): value and stage times.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --no-extras "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench_quick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print(d['value'], d['step_ms'], d['stages'], d['roofline']['frac'], d['host'])"
echo rc=0
