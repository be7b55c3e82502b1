#!/bin/bash
# round 5 session 22: sync step sums without the per-sample correlation zeroing: sync parity + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "sync" > gpurun_out/ab/par_sync.log 2>&1 || { echo "sync parity FAILED"; tail -30 gpurun_out/ab/par_sync.log; exit 1; }
echo "sync parity: $(tail -1 gpurun_out/ab/par_sync.log)"
NO_PMC=1 tools/ab_lib_pmc.sh base prev base prev 2>&1 | cut -c1-120
