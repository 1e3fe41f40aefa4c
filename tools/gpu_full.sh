export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench_full.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_full.json')); print(d['value'], d['stages'], json.dumps(d['extras']['c3j']))"
timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/probe_select.log 2>&1 || { echo PROBE_FAILED; exit 1; }
tail -14 gpurun_out/probe_select.log
