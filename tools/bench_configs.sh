#!/bin/bash
# bench.py on the other synthetic configs (C3 is
# bench.py's default), one GPU, full step definition, whole timed batch
# checked against the oracle.  Each run has its own time limit; the chain
# stops at the first failure.   bash tools/bench_configs.sh [C1 C2 C4 C5]
mkdir -p gpurun_out/configs
for c in ${@:-C1 C2 C4 C5}; do
  case $c in
    C1) args="--batch 1" ;;
    C2) args="--batch 1000" ;;
    C4) args="--batch 256" ;;
    C5) args="--batch 1024 --steps 20 --warmup 3 --cpu-sample 4" ;;
    *) echo "unknown config $c"; exit 2 ;;
  esac
  timeout -k 10 900 python bench.py --config $c $args --no-extras > gpurun_out/configs/$c.json 2> gpurun_out/configs/$c.err || exit 1
done
echo configs_done
