#!/bin/bash
# same-box A/B of an environment setting: `bash tools/ab_env.sh VAR v1 v2 ...` runs the short bench
# once per value (and the first value again at the end) and prints the per-kernel ms per chunk
set -e
var=$1; shift
mkdir -p gpurun_out
for v in "$@" "$1"; do
  env $var=$v timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 - "$var=$v" gpurun_out/ab_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d['kernel_ms_per_chunk']
print(sys.argv[1], d['value'], {n: round(k[n], 3) for n in k if k[n] > 0.1}, 'fec ok', d['check']['fec']['tb_crc_ok'])
PY
done
