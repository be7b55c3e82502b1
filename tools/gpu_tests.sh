#!/bin/bash
# GPU test pass on the box: every -m gpu test (no -x, so one failure does not hide the others),
# then smoke(). Logs under gpurun_out/.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | sed 's/ *\[.*//' | sort | uniq -c | sort -rn | head -5
grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -40
tail -3 gpurun_out/gpu_tests.log
exit $rc
