#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "tx_parity" --timeout 120 --timeout-method thread > gpurun_out/s3_tests.log 2>&1; rc=$?
tail -2 gpurun_out/s3_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s3_tests.log | head; exit $rc; }
DNRP_LIB=$PWD/dect-nr-plus-sdr_amd/libdnrp_fftswz.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "tx_parity or rx_parity" --timeout 120 --timeout-method thread > gpurun_out/s3_tests2.log 2>&1; rc=$?
tail -2 gpurun_out/s3_tests2.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s3_tests2.log | head; exit $rc; }
NO_PMC=1 tools/ab_lib_pmc.sh base tx_old fftswz base tx_old fftswz
tools/ab_lib_pmc.sh base fftswz
timeout -k 10 500 python tools/concur.py C4 16384
