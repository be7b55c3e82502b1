#!/bin/bash
# sync_peak with the STF region's input span staged in LDS (one load latency) vs direct loads
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -2
bash tools/ab_lib.sh default pkold default pkold
AB_ARGS="--workload C3" bash tools/ab.sh DNRP_RX_EPOCH=2 DNRP_RX_EPOCH=0 DNRP_RX_EPOCH=2 DNRP_RX_EPOCH=0
