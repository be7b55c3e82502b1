#!/bin/bash
# sync_post: STF staged in LDS + input-major FIR at 8 waves per SIMD (default) vs straight from the window (postold)
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -2
bash tools/ab_lib.sh default postold default postold
