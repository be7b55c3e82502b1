#!/bin/bash
# C3 device chunk A/B (pipelined)
set -e
mkdir -p gpurun_out
for c in 8192 16384 32768 8192 16384 32768; do
  timeout -k 10 300 python bench.py --workload C3 --steps 3 --no-cpu-baseline --chunk $c > gpurun_out/c3_$c.log 2>&1 || { tail -5 gpurun_out/c3_$c.log; exit 1; }
  python3 - $c gpurun_out/c3_$c.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print('C3 chunk', sys.argv[1], d['value'], d['ms_per_step'], d['serial_kernel_sum_ms_per_step'], d['config'].get('hbm_in_use_gb'), d['check']['fec']['tb_crc_ok'])
PY
done
