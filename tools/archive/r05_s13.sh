#!/bin/bash
# round 5 session 13: per-stream skew of the antenna-pair-interleaved pilot buffer (DNRP_ZFI_SKEW)
# against the rx_cells LDS conflicts -- RX parity of base and sk8, then time + LDS counters
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in base sk8; do
  if [ "$v" = base ]; then lib=$PWD/dect-nr-plus-sdr_amd/libdnrp.so; else lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so; fi
  DNRP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "rx_parity or sm_mmse" > gpurun_out/ab/par_$v.log 2>&1 || { echo "$v parity FAILED"; tail -20 gpurun_out/ab/par_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/ab/par_$v.log)"
done
tools/ab_lib_pmc.sh base sk4 sk8 sk16 2>&1 | grep -E "^(base|sk)|rx_cells|failed"
