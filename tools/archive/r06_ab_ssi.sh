#!/bin/bash
# sync_steps: FIR input-major (ssi, 131 VGPRs, 11 waves per CU by LDS) and with the 912-slot ring at
# 4 waves per SIMD (ssi912: 12 waves per CU) against the default (159 VGPRs, 1024 ring)
set -e
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_ssi912.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
bash tools/ab_lib.sh default ssi ssi912 default ssi ssi912
