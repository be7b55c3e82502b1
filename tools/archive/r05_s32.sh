#!/bin/bash
# round 5 session 32: RX front end staging and resampling stores branch-free (dead slot for elements
# outside the span or symbol): RX parity + A/B against the previous build
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "rx or loopback or chunk or fused or stride" > gpurun_out/ab/par_bf.log 2>&1 || { echo "rx parity FAILED"; tail -30 gpurun_out/ab/par_bf.log; exit 1; }
echo "rx parity: $(tail -1 gpurun_out/ab/par_bf.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base prev base prev 2>&1 | cut -c1-330
