#!/bin/bash
# A/B: PDC phase in packet groups over two streams (DNRP_RX_GROUP), Y re-read from the caches;
# parity of the grouped path on the bench chunk first (ragged last group).
set -e
mkdir -p gpurun_out/ab
DNRP_RX_GROUP=1000 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "full_chunk_edges and 16384" -x -q --timeout 240 --timeout-method thread 2>&1 | tail -3
AB_ARGS="${AB_ARGS}" bash tools/ab.sh "$@"
