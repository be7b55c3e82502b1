#!/bin/bash
# Kernel-trace stats + PMC passes for the bench (run on the GPU box from the repo root).
# Usage: tools/profile_r01.sh <tag> [bench args...]
set -e
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --no-cpu-baseline "$@" > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    --output-format csv -d $out/pmc_sq -o run -- python3 bench.py --no-cpu-baseline "$@" > $out/pmc_sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_FLAT \
    --output-format csv -d $out/pmc_sq2 -o run -- python3 bench.py --no-cpu-baseline "$@" > $out/pmc_sq2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- \
    python3 bench.py --no-cpu-baseline "$@" > $out/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- \
    python3 bench.py --no-cpu-baseline "$@" > $out/pmc_write.log 2>&1
rocprofv3 -L > $out/counters.txt 2>&1 || true
# keep the box output small: drop per-dispatch traces, keep only libdnrp rows of the PMC passes
rm -f $out/trace/run_kernel_trace.csv
for f in $out/pmc_*/run_counter_collection.csv; do
    python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keep = [r for r in rows if "dnrp" in r["Kernel_Name"]]
if rows:
    w = csv.DictWriter(open(sys.argv[1], "w", newline=""), fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(keep)
PY
done
