#!/bin/bash
# TX polyphase blocks: VALU (0) vs split-fp16 MFMA (1) vs f32 MFMA (2), same box; parity of the forms first
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "matrix_blocks" -x -q --timeout 240 --timeout-method thread 2>&1 | tail -2
bash tools/ab.sh DNRP_TX_MFMA=0 DNRP_TX_MFMA=2 DNRP_TX_MFMA=1 DNRP_TX_MFMA=0 DNRP_TX_MFMA=2
