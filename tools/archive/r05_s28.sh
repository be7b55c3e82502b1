#!/bin/bash
# round 5 session 28: C4SM line and PMC pass at its new 8192-slot chunk
set -e
export TMPDIR=/tmp
out=gpurun_out/final
mkdir -p $out
bash tools/profile_r03.sh r05_c4sm --workload C4SM --batch 8192
timeout -k 10 300 python bench.py --workload C4SM --no-cpu-baseline > $out/bench_c4sm.log 2>&1
grep '^{"metric"' $out/bench_c4sm.log | tail -1 > $out/bench_c4sm.json
python3 -c "import json; d=json.load(open('$out/bench_c4sm.json')); print(d['value'], d['ms_per_step'], d['serial_kernel_sum_ms_per_step'], d['kernel_ms_per_chunk']['rx_pdc'], d['config']['chunk'])"
