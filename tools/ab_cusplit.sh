#!/bin/bash
# A/B: sync stream restricted to K CUs (bench.py --cu-split K) against the unmasked streams
set -e
mkdir -p gpurun_out
for k in 0 32 64 0 16; do
  timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --cu-split $k > gpurun_out/cus_$k.log 2>&1 || { tail -5 gpurun_out/cus_$k.log; exit 1; }
  python3 - $k gpurun_out/cus_$k.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print('cu_split', sys.argv[1], d['value'], d['ms_per_step'], d['serial_kernel_sum_ms_per_step'], d['check']['sync_missed'], d['check']['fec']['tb_crc_ok'])
PY
done
