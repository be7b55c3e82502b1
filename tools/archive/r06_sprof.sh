#!/bin/bash
# sync_peak / sync_detect phase clocks (DNRP_SYNC_PROFILE build, wall_clock64 ticks of 10 ns)
set -e
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_sprof.so DNRP_SYNC_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --batch 16384 --no-cpu-baseline > gpurun_out/sprof.out 2> gpurun_out/sprof.err
grep -E "phases" gpurun_out/sprof.err | tail -4
