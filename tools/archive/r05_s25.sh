#!/bin/bash
# round 5 session 25: sync_fine's 4096-point transforms with compile-time passes and two butterflies
# per thread in flight (fft_r4_inplace_ct): sync parity + A/B against the previous build
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "sync or chunk" > gpurun_out/ab/par_fine.log 2>&1 || { echo "sync parity FAILED"; tail -30 gpurun_out/ab/par_fine.log; exit 1; }
echo "sync parity: $(tail -1 gpurun_out/ab/par_fine.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base prev base prev 2>&1 | cut -c1-330
