#!/bin/bash
# sync_steps segments, balanced: at most 64 chunks (default: 3 x 480 steps at C4) vs 32 (seg32: 5 x 288,
# the previous form), 96 (2 x 720), 160 (1 x 1440)
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_seg96.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
bash tools/ab_lib.sh default seg32 seg96 seg160 default seg32 seg96 seg160
