#!/bin/bash
# round 5 session 26: sync_peak segment sums and scans in one pass: sync parity, A/B against the
# previous build, and the phase clocks (DNRP_SYNC_PROFILE builds) of both
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "sync or chunk" > gpurun_out/ab/par_peak.log 2>&1 || { echo "sync parity FAILED"; tail -30 gpurun_out/ab/par_peak.log; exit 1; }
echo "sync parity: $(tail -1 gpurun_out/ab/par_peak.log)"
for v in prof prof2; do
  DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so DNRP_SYNC_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --batch 16384 --no-cpu-baseline > gpurun_out/ab/$v.out 2> gpurun_out/ab/$v.err || { echo "$v run failed"; tail -20 gpurun_out/ab/$v.err; exit 1; }
  echo "$v: $(grep -E 'sync_peak phases' gpurun_out/ab/$v.err | tail -1)"
  echo "$v: $(grep -E 'sync_detect phases' gpurun_out/ab/$v.err | tail -1)"
done
NO_PMC=1 tools/ab_lib_pmc.sh base prev base prev 2>&1 | cut -c1-330
