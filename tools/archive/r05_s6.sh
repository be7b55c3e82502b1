#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "rx_parity and not fused" --timeout 120 --timeout-method thread > gpurun_out/s6_tests.log 2>&1; rc=$?
tail -1 gpurun_out/s6_tests.log; [ $rc -ne 0 ] && exit $rc
NO_PMC=1 tools/ab_lib_pmc.sh base fe_nopf fe_spw4 fe_spw4_nopf base fe_nopf fe_spw4 fe_spw4_nopf
