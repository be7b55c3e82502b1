#!/bin/bash
# round 5 session 21: pilot-buffer build with the threads split by stream (DNRP_PILOTS_SPLIT): RX
# parity, then C4 and C4SM A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_psplit.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "rx or sm_mmse or chunk" > gpurun_out/ab/par_psplit.log 2>&1 || { echo "psplit parity FAILED"; tail -30 gpurun_out/ab/par_psplit.log; exit 1; }
echo "psplit parity: $(tail -1 gpurun_out/ab/par_psplit.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base psplit base psplit 2>&1 | cut -c1-260
AB_ARGS="--workload C4SM" NO_PMC=1 tools/ab_lib_pmc.sh base psplit 2>&1 | cut -c1-260
