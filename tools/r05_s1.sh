#!/bin/bash
# round-5 session 1: GPU tests, then the LDS-conflict attribution A/B
mkdir -p gpurun_out
tools/gpu_tests.sh > gpurun_out/s1_tests.txt 2>&1; rc=$?
cat gpurun_out/s1_tests.txt
[ $rc -ne 0 ] && exit $rc
tools/ab_lib_pmc.sh base cells_onerow cells_onewrow tx_noqtab
