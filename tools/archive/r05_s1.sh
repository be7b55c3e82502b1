#!/bin/bash
# round-5 session 1: GPU tests, then the LDS-conflict attribution A/B
mkdir -p gpurun_out
tools/gpu_tests.sh > gpurun_out/s1_tests.txt 2>&1; rc=$?
cat gpurun_out/s1_tests.txt
[ $rc -ne 0 ] && exit $rc
tools/ab_lib_pmc.sh base cells_onerow cells_onewrow tx_noqtab
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/s1_bench.log 2>&1 && tail -1 gpurun_out/s1_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['value'], d['ms_per_step'], d['serial_kernel_sum_ms_per_step'])"
