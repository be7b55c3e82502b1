#!/bin/bash
# rx_cells: pilot sources issued before the weight-table staging (default) vs build_pilots after it (cpp0);
# C4 (PCC phase) and C4SM (MMSE PDC phase through rx_cells)
set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
bash tools/ab_lib.sh default cpp0 default cpp0
AB_ARGS="--workload C4SM" bash tools/ab_lib.sh default cpp0 default cpp0
