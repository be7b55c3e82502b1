#!/bin/bash
# A/B of the device chunk (slots per launch), pipelined and one-stream
set -e
mkdir -p gpurun_out
for c in 4096 8192 16384 4096; do
  for ser in 0 1; do
    DNRP_BENCH_SERIAL=$ser timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --chunk $c > gpurun_out/chunk_${c}_$ser.log 2>&1 || { tail -5 gpurun_out/chunk_${c}_$ser.log; exit 1; }
    python3 - $c $ser gpurun_out/chunk_${c}_$ser.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print('chunk', sys.argv[1], 'serial', sys.argv[2], d['value'], d['ms_per_step'], d['serial_kernel_sum_ms_per_step'], d['check']['fec']['tb_crc_ok'])
PY
  done
done
