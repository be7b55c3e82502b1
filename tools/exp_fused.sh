#!/bin/bash
# Phase-skip builds of the fused PDC receiver (tools/build_variant.sh skipeq / skipfe / skipboth) vs
# the default, same box: per-chunk kernel times of a 3-step bench.
mkdir -p gpurun_out
for v in default skipeq skipfe skipboth default; do
  lib=""; [ $v != default ] && lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so
  DNRP_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/exp_$v.log 2>&1 || { tail -5 gpurun_out/exp_$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/exp_{sys.argv[1]}.log').read().strip().splitlines()[-1])
k = d['kernel_ms_per_chunk']
print(sys.argv[1], d['value'], 'fused', k.get('rx_fused'), 'fft_pdc', k.get('rx_fft_pdc'), 'pdc', k.get('rx_pdc'))
PY
done
