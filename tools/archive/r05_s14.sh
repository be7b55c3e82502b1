#!/bin/bash
# round 5 session 14: TX bins from per-stream one-hot code tables (kernels.hpp OH_*): TX parity, then
# TX alone and the C4 bench against the previous build
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "tx or loopback or fec or full_chunk" > gpurun_out/ab/par_oh.log 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/ab/par_oh.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/ab/par_oh.log)"
for v in prev base prev base; do
  if [ "$v" = base ]; then lib=$PWD/dect-nr-plus-sdr_amd/libdnrp.so; else lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so; fi
  echo "$v $(DNRP_LIB=$lib timeout -k 10 200 python tools/tx_time.py C4 16384 5)" || exit 1
done
NO_PMC=1 tools/ab_lib_pmc.sh base prev
