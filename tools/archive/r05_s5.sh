#!/bin/bash
mkdir -p gpurun_out
for w in C4 C3; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --workload $w > gpurun_out/s5_$w.log 2>&1 || { tail -5 gpurun_out/s5_$w.log; exit 1; }
  tail -1 gpurun_out/s5_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['value'], d['ms_per_step'], d['serial_kernel_sum_ms_per_step'], {k: round(v,2) for k,v in d['kernel_ms_per_chunk'].items()})"
done
