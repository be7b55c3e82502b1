#!/bin/bash
# sync_fine: radix-8 4096-point transforms at 8 waves per SIMD (default, spills), radix 8 at the
# compiler's occupancy (r8w4), radix 4 (r4, the previous default)
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -2
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_r8w4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
bash tools/ab_lib.sh default r8w4 r4 default r8w4 r4
