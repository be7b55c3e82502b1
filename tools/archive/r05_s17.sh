#!/bin/bash
# round 5 session 17: FE amplitude folded into the derotation phasors (DNRP_FE_BINS_FOLD): RX parity + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_fefold.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "rx or sync_then" > gpurun_out/ab/par_fefold.log 2>&1 || { echo "fefold parity FAILED"; tail -30 gpurun_out/ab/par_fefold.log; exit 1; }
echo "fefold parity: $(tail -1 gpurun_out/ab/par_fefold.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base fefold base fefold
