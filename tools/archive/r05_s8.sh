#!/bin/bash
# round 5 session 8: MMSE interpolation chunking + MFMA Gram A/B (C4SM) with parity first
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
ok=""
for v in mm2 mm3 mmfma; do
  if DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -k "sm_mmse" > gpurun_out/ab/par_$v.log 2>&1; then
    ok="$ok $v"; echo "$v parity: $(tail -1 gpurun_out/ab/par_$v.log)"
  else
    rc=$?; echo "$v parity FAILED rc=$rc"; tail -25 gpurun_out/ab/par_$v.log
    case $rc in 124|134|137|139) exit 1;; esac
  fi
done
AB_ARGS="--workload C4SM" tools/ab_lib_pmc.sh base $ok
