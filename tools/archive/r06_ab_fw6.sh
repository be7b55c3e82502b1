#!/bin/bash
# sync_fine at 6 waves per SIMD (3 workgroups per CU, 80 VGPRs + 76 B spills) vs the compiler's 113 VGPRs (2)
set -e
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_fw6.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
bash tools/ab_lib.sh default fw6 default fw6
