#!/bin/bash
# rx_stf_ant: FIR input-major from LDS at 8 waves per SIMD (default) vs the window in registers (stfold)
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "rx" 2>&1 | tail -2
bash tools/ab_lib.sh default stfold default stfold
