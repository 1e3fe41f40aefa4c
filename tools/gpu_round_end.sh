#!/bin/bash
# Round-end evidence in one box: tools/gpu_final.sh (tests, full C3 bench,
# rocprof, PMC, probes), then every other config (tools/bench_configs.sh).
bash tools/gpu_final.sh || exit 1
bash tools/bench_configs.sh || { echo CONFIGS_FAILED; exit 1; }
for c in C1 C2 C4 C5; do python -c "import json,sys; d=json.load(open('gpurun_out/configs/$c.json')); print('$c', d['value'], d['step_ms']['median'], d['parity_full_batch']['ok'])"; done
echo round_end_done
