#!/bin/bash
# round 5 session 15: TX bin cost left (trivial-bins probe) and the OHX bins variant (parity + time)
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_ohx.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "tx" > gpurun_out/ab/par_ohx.log 2>&1 || { echo "ohx parity FAILED"; tail -30 gpurun_out/ab/par_ohx.log; }
echo "ohx parity: $(tail -1 gpurun_out/ab/par_ohx.log)"
for v in base txtb ohx base ohx; do
  if [ "$v" = base ]; then lib=$PWD/dect-nr-plus-sdr_amd/libdnrp.so; else lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so; fi
  echo "$v $(DNRP_LIB=$lib timeout -k 10 200 python tools/tx_time.py C4 16384 5)" || exit 1
done
