#!/bin/bash
# rx_stf_kernel: STF cells of every antenna and the STF values staged in one load round (default) vs the
# per-antenna loop and per-call STF reads (stfk0)
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sync.py -x -q --timeout 240 --timeout-method thread -k "rx or sync" 2>&1 | tail -1
bash tools/ab_lib.sh default stfk0 default stfk0
