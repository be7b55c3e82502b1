#!/bin/bash
# PC sampling probe (rocprofv3 beta) of the TX kernel alone: where its waves sit
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
timeout -s KILL 150 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1; grep -i -A12 "pc sampling\|pc_sampling" gpurun_out/pcs/list.txt | head -40
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --output-format csv -d gpurun_out/pcs/st -o run -- python3 tools/tx_time.py C4 4096 2 > gpurun_out/pcs/st.log 2>&1; echo "stochastic rc=$?"; tail -3 gpurun_out/pcs/st.log
ls -R gpurun_out/pcs | head -20
