#!/bin/bash
# TX on the GPU: every TX parity test, then the short bench (per-kernel ms per 4096-slot chunk)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "tx" -q --timeout 120 --timeout-method thread > gpurun_out/tx_tests.log 2>&1 || { tail -30 gpurun_out/tx_tests.log; exit 1; }
tail -1 gpurun_out/tx_tests.log
bash tools/ab_env.sh DNRP_NONE 0
