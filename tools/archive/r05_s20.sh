#!/bin/bash
# round 5 session 20: experiment alternatives' parity (tools/r05_s19.sh), then the real-W TX bins
# variant (DNRP_TX_REALW): TX parity and TX time against the base build
export TMPDIR=/tmp
bash tools/r05_s19.sh || exit 1
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_realw.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q \
    --timeout 120 --timeout-method thread -k "tx_parity" > gpurun_out/xs/par_realw.log 2>&1; echo "realw parity rc=$? $(tail -1 gpurun_out/xs/par_realw.log)"
for v in base realw base realw; do
  if [ "$v" = base ]; then lib=$PWD/dect-nr-plus-sdr_amd/libdnrp.so; else lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so; fi
  echo "$v $(DNRP_LIB=$lib timeout -k 10 200 python tools/tx_time.py C4 16384 5)" || exit 1
done
