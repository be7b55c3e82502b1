#!/bin/bash
# Round-4 fused PDC receiver check on the GPU box: RX parity tests (fused default + the new cases),
# then the bench with the fused receiver and with the Y path (DNRP_RX_FUSED=0) on the same box.
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "rx" -q --timeout 120 --timeout-method thread "$@" > gpurun_out/rx_tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/rx_tests.log | head -30; tail -3 gpurun_out/rx_tests.log; exit 1; }
tail -2 gpurun_out/rx_tests.log
for v in 1 0 1; do
  DNRP_RX_FUSED=$v timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/bench_fused$v.log 2>&1 || { tail -5 gpurun_out/bench_fused$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/bench_fused{sys.argv[1]}.log').read().strip().splitlines()[-1])
print("fused", sys.argv[1], d['value'], {k: round(v, 3) for k, v in d['kernel_ms_per_chunk'].items()}, d['check']['fec'], d['roofline'], d['hbm'])
PY
done
