#!/bin/bash
# polyphase windows input-major from LDS (pp_const::run_imaj) in TX (default) vs loaded whole (txi0),
# in the RX front end (default) vs loaded whole (fei0); sync_steps step-sum reads 16 in flight (ssg16)
set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_stream.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -1
bash tools/ab_lib.sh default txi0 fei0 ssg16 default txi0 fei0 ssg16
