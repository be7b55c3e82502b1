#!/bin/bash
# round 5 session 33: RX front end resampling stores branch-free (outputs outside the symbol to
# per-lane dead slots; staging unchanged): RX parity + A/B against the previous build
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "rx or loopback or chunk or fused or stride" > gpurun_out/ab/par_bf2.log 2>&1 || { echo "rx parity FAILED"; tail -30 gpurun_out/ab/par_bf2.log; exit 1; }
echo "rx parity: $(tail -1 gpurun_out/ab/par_bf2.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base prev base prev 2>&1 | cut -c1-330
