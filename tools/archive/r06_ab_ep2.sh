#!/bin/bash
# epoch receiver A/B: nontemporal Y stores / antenna-major front-end tasks
set -e
for v in epnt epam epamnt; do
  DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "epoch and (C4 or tm5 or lmode)" -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
done
bash tools/ab_lib.sh default epnt epam epamnt default
