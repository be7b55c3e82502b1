#!/bin/bash
# FEC GPU tests + encode timing
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_fec.py -q --timeout 240 --timeout-method thread 2>&1 | tail -4
timeout -k 10 200 python tools/bench_fec_enc.py --n 16384 2>&1 | tail -1
