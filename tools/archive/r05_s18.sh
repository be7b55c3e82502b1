#!/bin/bash
# round 5 session 18: zero-padded LDS weight rows (no clamps / selects in the equaliser taps): RX
# parity (every RX case incl. strides, MRC, MMSE, fused, chunk edges), then C4 + C4SM A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "rx or sm_mmse or chunk or sync_then or loopback or fec" > gpurun_out/ab/par_wpad.log 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/ab/par_wpad.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/ab/par_wpad.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base prev base prev
AB_ARGS="--workload C4SM" NO_PMC=1 tools/ab_lib_pmc.sh base prev
