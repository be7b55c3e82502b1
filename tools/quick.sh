#!/bin/bash
# quick GPU check: sync + parity tests, short bench; prints per-kernel ms per 4096-slot launch
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1])
print(d['value'], {k: round(v, 2) for k, v in d['kernel_ms_per_chunk'].items()}, d['check'])
PY
