#!/bin/bash
# rx_epoch: pilot sources, segment descriptors and LUT picks loaded before the phase barrier (default)
# vs after it (pf0)
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "rx" 2>&1 | tail -1
bash tools/ab_lib.sh default pf0 default pf0
