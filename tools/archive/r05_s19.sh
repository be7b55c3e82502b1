#!/bin/bash
# round 5 session 19: the measured-alternative experiment bits still compute the product's results
# (XS_WFFT_SWZ 16384, XS_TX_QLEV 32768, XS_FE_PREFETCH 65536, XS_MMSE_MFMA 131072)
export TMPDIR=/tmp
mkdir -p gpurun_out/xs
for v in 16384:"tx_parity or rx_parity" 32768:"tx_parity" 65536:"rx_parity" 131072:"sm_mmse"; do
  b=${v%%:*}; k=${v#*:}
  DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_xs$b.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q \
      --timeout 120 --timeout-method thread -k "$k" > gpurun_out/xs/par_$b.log 2>&1
  rc=$?; echo "xs$b ($k): rc=$rc $(tail -1 gpurun_out/xs/par_$b.log)"
  case $rc in 124|134|137|139) exit 1;; esac
done
