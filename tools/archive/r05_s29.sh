#!/bin/bash
# round 5 session 29: the C4SM line again, now that profiles/r05 holds its 8192-slot PMC summaries
set -e
export TMPDIR=/tmp
out=gpurun_out/final
mkdir -p $out
timeout -k 10 300 python bench.py --workload C4SM --no-cpu-baseline > $out/bench_c4sm.log 2>&1
grep '^{"metric"' $out/bench_c4sm.log | tail -1 > $out/bench_c4sm.json
python3 -c "import json; d=json.load(open('$out/bench_c4sm.json')); print(d['value'], d['ms_per_step'], d['serial_kernel_sum_ms_per_step'], d['kernel_ms_per_chunk']['rx_pdc'], d['roofline'], d.get('roofline_valu'))"
