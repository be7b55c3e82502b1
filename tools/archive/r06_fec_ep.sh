#!/bin/bash
# FEC encoder rewrite: GPU FEC tests + encode timing; epoch receiver phase-skip builds.
set -e
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_fec.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -4
timeout -k 10 200 python tools/bench_fec_enc.py --n 16384 2>&1 | tail -2
DNRP_RX_EPOCH=1 bash tools/ab_lib.sh default epskipfe epskipeq epskipboth
