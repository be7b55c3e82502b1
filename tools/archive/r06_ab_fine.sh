#!/bin/bash
# sync_fine: spectrum x template loads batched 8 per thread (default) vs one per loop iteration (fine1)
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -2
bash tools/ab_lib.sh default fine1 default fine1
