#!/bin/bash
# sync_steps: 912-slot ring with a 32-bit modulo (12 waves per CU by LDS) vs the 1024 ring (11)
set -e
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_ss912.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
bash tools/ab_lib.sh default ss912 default ss912
