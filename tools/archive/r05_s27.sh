#!/bin/bash
# round 5 session 27: device chunk size of the C4SM and C3 lines (A/B, same box)
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
run() {  # workload chunk tag
  timeout -k 10 300 python bench.py --workload $1 --chunk $2 --no-cpu-baseline > gpurun_out/ab/ch_$3.log 2>&1 || { echo "$3 failed"; tail -5 gpurun_out/ab/ch_$3.log; exit 1; }
  python3 - "$3" "gpurun_out/ab/ch_$3.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]).read().splitlines() if l.startswith('{"metric"')][-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d.get('serial_kernel_sum_ms_per_step'), d['config'].get('hbm_in_use_gb'), flush=True)
PY
}
run C4SM 4096 sm4k && run C4SM 8192 sm8k && run C4SM 4096 sm4k_2 && run C4SM 8192 sm8k_2 && \
run C3 8192 c3_8k && run C3 16384 c3_16k && run C3 8192 c3_8k_2 && run C3 16384 c3_16k_2
