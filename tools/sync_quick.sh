#!/bin/bash
# sync kernels on the GPU: every sync test, then a short bench (per-kernel ms per 4096-slot chunk)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/sync_tests.log 2>&1 || { tail -30 gpurun_out/sync_tests.log; exit 1; }
tail -1 gpurun_out/sync_tests.log
timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1])
print(d['value'], {k: round(v, 3) for k, v in d['kernel_ms_per_chunk'].items()}, d['check'])
PY
