#!/bin/bash
# round 5 session 24: 256-QAM one-hot codes with staging-relative byte indices: TX parity + TX A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "tx or loopback or chunk or fec" > gpurun_out/ab/par_rel.log 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/ab/par_rel.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/ab/par_rel.log)"
for v in prev base prev base; do
  if [ "$v" = base ]; then lib=$PWD/dect-nr-plus-sdr_amd/libdnrp.so; else lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so; fi
  echo "$v $(DNRP_LIB=$lib timeout -k 10 200 python tools/tx_time.py C4 16384 5)" || exit 1
done
