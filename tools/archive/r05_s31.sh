#!/bin/bash
# round 5 session 31: RX front end with the static bin map of beta = 16 (no per-bin range tests or
# phasor selects): RX parity + A/B against the previous build
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "rx or loopback or chunk or fused or stride" > gpurun_out/ab/par_bins.log 2>&1 || { echo "rx parity FAILED"; tail -30 gpurun_out/ab/par_bins.log; exit 1; }
echo "rx parity: $(tail -1 gpurun_out/ab/par_bins.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base prev base prev 2>&1 | cut -c1-330
