#!/bin/bash
# span staging in one round trip: sync_peak / sync_post 11 loads per thread (default) vs 6 (stg6);
# rx_stf_ant 10 (default) vs 8 (stfu8)
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "rx" 2>&1 | tail -1
bash tools/ab_lib.sh default stg6 stfu8 default stg6 stfu8
