#!/bin/bash
# round 5 session 23: padded lookback ring for the sync step sums (DNRP_SS_PADRING): sync parity + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_padring.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "sync" > gpurun_out/ab/par_padring.log 2>&1 || { echo "padring parity FAILED"; tail -30 gpurun_out/ab/par_padring.log; exit 1; }
echo "padring parity: $(tail -1 gpurun_out/ab/par_padring.log)"
tools/ab_lib_pmc.sh base padring 2>&1 | grep -E "^(base|padring)|sync_steps" | cut -c1-230
NO_PMC=1 tools/ab_lib_pmc.sh base padring 2>&1 | cut -c1-120
