#!/bin/bash
# A/B of library builds on one box: tools/ab_lib.sh name1 name2 ... (dect-nr-plus-sdr_amd/libdnrp_<name>.so,
# "default" = libdnrp.so), each a 3-step bench; prints value and the per-chunk kernel times.
mkdir -p gpurun_out
for v in "$@"; do
  lib=""; [ $v != default ] && lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so
  DNRP_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline $AB_ARGS > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/ab_{sys.argv[1]}.log').read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], {k: round(v, 3) for k, v in d['kernel_ms_per_chunk'].items() if v})
PY
done
