#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/exp_knobs.sh KUEUE_TAS_HOST_PIN 0 1 0 1 || exit 1
KUEUE_TAS_HOST_PIN=0 timeout -k 10 120 python tools/probe_trace.py C3 > gpurun_out/trace_pin0.log 2>&1 && tail -7 gpurun_out/trace_pin0.log
KUEUE_TAS_HOST_PIN=1 timeout -k 10 120 python tools/probe_trace.py C3 > gpurun_out/trace_pin1.log 2>&1 && tail -7 gpurun_out/trace_pin1.log
bash tools/gpu_pcie_exp.sh
