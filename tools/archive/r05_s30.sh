#!/bin/bash
# round 5 session 30: sync_peak resampling with each lane's own 10 inputs loaded and the rest of its
# window from lanes +1..+3 by DPP wave shifts: sync parity + A/B against the previous build
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "sync or chunk" > gpurun_out/ab/par_dpp.log 2>&1 || { echo "sync parity FAILED"; tail -30 gpurun_out/ab/par_dpp.log; exit 1; }
echo "sync parity: $(tail -1 gpurun_out/ab/par_dpp.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base prev base prev 2>&1 | cut -c1-330
