#!/bin/bash
# Which fast-LFC kernel stalls the BestFit select?  KTAS_DEBUG_LFC_ORDER
# moves the branch's last kernels after the BestFit select (1: lfc_emit,
# 2: + its select, 3: the whole branch); per-eval ticks each way.
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 2 3; do
  KTAS_DEBUG_LFC_ORDER=$m timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/sel_order$m.log 2>&1 || { echo S${m}_FAILED; exit 1; }
done
echo rc=0
