#!/bin/bash
# A/B of an experiment knob (env var $1 over the values $2...) on the C3
# bench without the CPU legs: step time and stage times per value.
export TMPDIR=/tmp
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 100 --warmup 20 > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.err || { echo "EXP_FAILED $v"; tail -3 gpurun_out/exp_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/exp_$v.json')); print('$var=$v', d['value'], d['ms_per_step'], d['step_ms']['median'], d['stages'])"
done
echo rc=0
