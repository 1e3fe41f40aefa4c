#!/bin/bash
# Is the BestFit select's final-walk stall PCIe contention with the fast-LFC
# emit's writes to mapped host memory?  Per-eval select profile with the
# default path, without device Values tags (host Values), and with the emit's
# stores skipped (diagnostic: results not used).
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "default::" "host_values:HOST_VALUES=1:" "no_emit_writes::1"; do
  name=${v%%:*}; rest=${v#*:}; hv=${rest%%:*}; ef=${rest#*:}
  env $hv KTAS_EXP_FLAGS=${ef:-0} timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/pcie_$name.log 2>&1 || { echo "PROBE_FAILED $name"; tail gpurun_out/pcie_$name.log; exit 1; }
  echo "== $name"; head -3 gpurun_out/pcie_$name.log | cut -c1-400; tail -11 gpurun_out/pcie_$name.log
done
echo rc=0
