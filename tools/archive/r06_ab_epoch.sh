#!/bin/bash
# Epoch receiver: parity first (every epoch case + the bench chunk), then the bench A/B.
set -e
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "epoch" -x -q --timeout 240 --timeout-method thread 2>&1 | tail -4
bash tools/ab.sh "$@"
