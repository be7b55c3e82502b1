#!/bin/bash
# sync_steps occupancy A/B (lazy FIR window + 4-sample step-sum groups: 126 VGPRs; 912-slot ring):
# sync parity on the default build, then the bench per library build.
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -3
bash tools/ab_lib.sh default ssv0 ssv1 default ssv0
