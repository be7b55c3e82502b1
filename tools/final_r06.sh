#!/bin/bash
# Round-6 measurement on the GPU box: every -m gpu test, smoke(), the default bench line (with the CPU
# baseline), the C4SM (MMSE) and C3 lines, and the default bench under rocprofv3 --kernel-trace --stats
# with the per-grid split of its closing one-stream step. Results -> gpurun_out/final6/
set -e
out=gpurun_out/final6
mkdir -p $out
export TMPDIR=/tmp
export DNRP_PARITY_STATS=$PWD/$out/parity_stats.jsonl
rm -f $DNRP_PARITY_STATS
bash tools/gpu_tests.sh
cp gpurun_out/gpu_tests.log $out/gpu_tests.log
unset DNRP_PARITY_STATS
timeout -k 10 200 python tools/bench_fec_enc.py --n 16384 > $out/fec_enc.json 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1
grep '^{"metric"' $out/bench_default.log | tail -1 > $out/bench_c4_default.json
timeout -k 10 300 python bench.py --workload C4SM --no-cpu-baseline > $out/bench_c4sm.log 2>&1
grep '^{"metric"' $out/bench_c4sm.log | tail -1 > $out/bench_c4sm.json
timeout -k 10 300 python bench.py --workload C3 --no-cpu-baseline > $out/bench_c3.log 2>&1
grep '^{"metric"' $out/bench_c3.log | tail -1 > $out/bench_c3.json
timeout -k 10 300 python bench.py --workload C2 --steps 200 --no-cpu-baseline > $out/bench_c2.log 2>&1
grep '^{"metric"' $out/bench_c2.log | tail -1 > $out/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu-baseline > $out/bench_rocprof.log 2>&1
grep '^{"metric"' $out/bench_rocprof.log | tail -1 > $out/bench_c4_under_rocprof.json
stats=$(find $out/trace -name "*kernel_stats.csv" | head -1)
trace=$(find $out/trace -name "*kernel_trace.csv" | head -1)
cp $stats $out/kernel_stats_c4_default_bench.csv
python3 tools/trace_by_grid.py $trace --tail 4 > $out/kernel_by_grid_c4_default_serial_step.txt
python3 tools/trace_by_grid.py $trace > $out/kernel_by_grid_c4_default_all.txt
rm -rf $out/trace
head -20 $out/kernel_by_grid_c4_default_serial_step.txt
python3 - <<'PY'
import json
for f in ("bench_c4_default", "bench_c4sm", "bench_c3", "bench_c2"):
    d = json.loads(open(f'gpurun_out/final6/{f}.json').read())
    print(f, d['value'], d['roofline'], d.get('hbm'), d.get('cpu_baseline', {}).get('value'), d['check']['fec'])
PY
