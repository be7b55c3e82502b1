#!/bin/bash
# A/B of environment switches on the bench: tools/ab.sh "VAR=a" "VAR=b" ... -> per-kernel ms per 4096-slot chunk
# (AB_ARGS: extra bench.py arguments, e.g. AB_ARGS="--workload C3")
mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline $AB_ARGS > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], {k: round(v, 2) for k, v in d['kernel_ms_per_chunk'].items()}, 'ber', round(d['check']['pdc_hard_ber'], 6))
PY
done
