export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/probe_select.log 2>&1 || { echo PROBE_FAILED; tail gpurun_out/probe_select.log; exit 1; }
head -6 gpurun_out/probe_select.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['i'], d['us'], d['cls'], d['count'], d['prof_us'])"
tail -12 gpurun_out/probe_select.log
