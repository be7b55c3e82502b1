#!/bin/bash
# split sync_detect at 7 waves per SIMD (default) vs 3 (detold); sync_peak windows input-major (default) vs loaded whole (pkim0)
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -2
bash tools/ab_lib.sh default detold pkim0 default detold pkim0
