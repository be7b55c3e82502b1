#!/bin/bash
# Round-5 measurement on the GPU box: every -m gpu test, smoke(), the default bench line (with the CPU
# baseline), the C4SM (MMSE) and C3 lines, and the default bench under rocprofv3 --kernel-trace --stats
# with the per-grid split of its closing one-stream step. Results -> gpurun_out/final/
set -e
out=gpurun_out/final
mkdir -p $out
export TMPDIR=/tmp
bash tools/gpu_tests.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1
grep '^{"metric"' $out/bench_default.log | tail -1 > $out/bench_c4_default.json
timeout -k 10 300 python bench.py --workload C4SM --no-cpu-baseline > $out/bench_c4sm.log 2>&1
grep '^{"metric"' $out/bench_c4sm.log | tail -1 > $out/bench_c4sm.json
timeout -k 10 300 python bench.py --workload C3 --no-cpu-baseline > $out/bench_c3.log 2>&1
grep '^{"metric"' $out/bench_c3.log | tail -1 > $out/bench_c3.json
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
for f in ("bench_c4_default", "bench_c4sm", "bench_c3"):
    d = json.loads(open(f'gpurun_out/final/{f}.json').read())
    print(f, d['value'], d['roofline'], d.get('hbm'), d.get('cpu_baseline', {}).get('value'), d['check']['fec'])
PY
