#!/bin/bash
# sync_peak at 6 waves per SIMD (3 workgroups per CU, 80 VGPRs + spills), staged span, window from LDS as consumed (pk6) or loaded whole (pk6d)
set -e
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_pk6.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -2
bash tools/ab_lib.sh default pk6 pk6d default pk6 pk6d
