#!/bin/bash
# bench.py on every synthetic config, one GPU; each run has
# its own time limit and the chain stops at the first failure.
mkdir -p gpurun_out/configs
timeout -k 10 300 python bench.py --config C3 > gpurun_out/configs/C3.json 2> gpurun_out/configs/C3.err || exit 1
timeout -k 10 300 python bench.py --config C1 --batch 1 > gpurun_out/configs/C1.json 2> gpurun_out/configs/C1.err || exit 1
timeout -k 10 300 python bench.py --config C2 --batch 1000 > gpurun_out/configs/C2.json 2> gpurun_out/configs/C2.err || exit 1
timeout -k 10 300 python bench.py --config C4 --batch 256 > gpurun_out/configs/C4.json 2> gpurun_out/configs/C4.err || exit 1
KTAS_CPU_THREADS=8 timeout -k 10 600 python bench.py --config C5 --batch 256 --steps 20 --warmup 3 --cpu-sample 4 --parity-sample 4 > gpurun_out/configs/C5.json 2> gpurun_out/configs/C5.err || exit 1
echo configs_done
