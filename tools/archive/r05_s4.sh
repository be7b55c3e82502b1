#!/bin/bash
mkdir -p gpurun_out
for r in 1 2; do for v in base tx_old txqlev; do
  if [ $v = base ]; then lib=$PWD/dect-nr-plus-sdr_amd/libdnrp.so; else lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so; fi
  TAG=$v DNRP_LIB=$lib timeout -k 10 200 python tools/tx_time.py C4 16384 5 || exit 1
done; done
DNRP_TIMING=0 timeout -k 10 500 python tools/concur.py C4 16384 || exit 1
DNRP_TIMING=1 timeout -k 10 500 python tools/concur.py C4 16384
