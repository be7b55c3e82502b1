#!/bin/bash
# round 5 session 16: sync look-ahead depth of the bench pipeline (DNRP_BENCH_AHEAD 1 vs 2), C3 and
# C4 lines back to back on one box; TX parity of the closing one-hot bins
export TMPDIR=/tmp
mkdir -p gpurun_out/ahead
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tx" \
    > gpurun_out/ahead/par_tx.log 2>&1 || { echo "TX parity FAILED"; tail -20 gpurun_out/ahead/par_tx.log; exit 1; }
echo "TX parity: $(tail -1 gpurun_out/ahead/par_tx.log)"
for wl in C3 C4; do
  for a in 1 2 1 2; do
    DNRP_BENCH_AHEAD=$a timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/ahead/${wl}_$a.log 2>&1 || { echo "$wl $a failed"; tail -5 gpurun_out/ahead/${wl}_$a.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ahead/${wl}_$a.log').read().strip().splitlines()[-1])
print('$wl ahead=$a', d['value'], 'ms/step', d['ms_per_step'], 'serial', d['serial_kernel_sum_ms_per_step'])"
  done
done
