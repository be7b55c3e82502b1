#!/bin/bash
# round 5 session 9: MMSE VALU diet (interleaved pilots, compiled demap width, packed int16) parity + C4SM A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "sm_mmse or rx_parity or fec" > gpurun_out/ab/par_base.log 2>&1 || { echo "base parity FAILED"; tail -30 gpurun_out/ab/par_base.log; exit 1; }
echo "base parity: $(tail -1 gpurun_out/ab/par_base.log)"
ok="base prev"
if false && DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_mmfma.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "sm_mmse" > gpurun_out/ab/par_mmfma.log 2>&1; then
  ok="$ok mmfma"; echo "mmfma parity: $(tail -1 gpurun_out/ab/par_mmfma.log)"
else
  rc=$?; echo "mmfma parity FAILED rc=$rc"; tail -25 gpurun_out/ab/par_mmfma.log
  case $rc in 124|134|137|139) exit 1;; esac
fi
AB_ARGS="--workload C4SM" tools/ab_lib_pmc.sh $ok
