#!/bin/bash
# round 5 session 10: SFBC pilot pairs + LLR packing: RX parity, then C4 A/B (base vs prev)
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "rx or sm_mmse or fec or chunk" > gpurun_out/ab/par_base.log 2>&1 || { echo "base parity FAILED"; tail -30 gpurun_out/ab/par_base.log; exit 1; }
echo "base parity: $(tail -1 gpurun_out/ab/par_base.log)"
tools/ab_lib_pmc.sh base prev
