#!/bin/bash
# round 5 session 12: persistent-grid TX (capped workgroups per CU) -- TX alone and next to sync_steps
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in prev base tp2 tp1; do
  if [ "$v" = base ]; then lib=$PWD/dect-nr-plus-sdr_amd/libdnrp.so; else lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so; fi
  echo "== $v"
  DNRP_LIB=$lib timeout -k 10 200 python tools/tx_time.py C4 16384 5 || exit 1
  DNRP_LIB=$lib timeout -k 10 300 python tools/concur.py C4 16384 > gpurun_out/ab/conc_$v.log 2>&1 || { tail -5 gpurun_out/ab/conc_$v.log; exit 1; }
  grep '^{' gpurun_out/ab/conc_$v.log | tail -1
done
