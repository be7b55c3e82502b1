#!/bin/bash
# Round-6 full check: every -m gpu test (LLR-gate statistics recorded), FEC encode timing, smoke(),
# the default bench line. -> gpurun_out/r06/
set -e
out=gpurun_out/r06
mkdir -p $out
export TMPDIR=/tmp
export DNRP_PARITY_STATS=$PWD/$out/parity_stats.jsonl
rm -f $DNRP_PARITY_STATS
bash tools/gpu_tests.sh || echo "GPU TESTS FAILED"
cp gpurun_out/gpu_tests.log $out/gpu_tests.log
unset DNRP_PARITY_STATS
timeout -k 10 200 python tools/bench_fec_enc.py --n 16384 2>&1 | tail -1 | tee $out/fec_enc.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $out/bench.log 2>&1
grep '^{"metric"' $out/bench.log | tail -1 > $out/bench.json
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/r06/bench.json').read())
print(d['value'], d['roofline'], {k: v for k, v in d['kernel_ms_per_chunk'].items() if v}, d['check']['fec'])
PY
