#!/bin/bash
# round-5 session 2: RX parity tests on the rx_cells rewrite, then the A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "rx_parity or chunk_edges or largest or grow" --timeout 120 --timeout-method thread > gpurun_out/s2_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s2_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s2_tests.log | head; exit $rc; }
NO_PMC=1 tools/ab_lib_pmc.sh base cells_old cells_ch2 base cells_old
tools/ab_lib_pmc.sh base
