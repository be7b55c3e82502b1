#!/bin/bash
# sync_peak metric: uniform doubles in SGPRs + per-slide addresses (default, 20 B spills) vs 88 B (psr0);
# rx_stf_kernel's packet state in registers (no scratch struct)
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "rx" 2>&1 | tail -1
bash tools/ab_lib.sh default psr0 default psr0
