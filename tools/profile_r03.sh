#!/bin/bash
# Round-3 profile of one bench step (C4, one 4096-slot chunk unless args override): kernel-trace stats
# and per-kernel PMC passes (SQ wave-cycle split + instruction mix, LDS, FETCH_SIZE, WRITE_SIZE),
# each pass its own run (gfx950 slot limits, MI355X_MICROARCH.md). Summaries -> gpurun_out/prof_<tag>/
set -e
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
args="--no-cpu-baseline --steps 1 --warmup 0 --batch 4096 $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args > $out/trace.log 2>&1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 bench.py $args > $out/p$i.log 2>&1
done
python3 tools/pmc_r02_summary.py $out > $out/summary.txt
# FETCH_SIZE / WRITE_SIZE per launch -> traffic.json (tools/traffic_summary.py layout)
mkdir -p $out/pmc_fetch $out/pmc_write $out/pmc_valu
mv $(find $out/p3 -name "*counter_collection.csv" | head -1) $out/pmc_fetch/run_counter_collection.csv
mv $(find $out/p4 -name "*counter_collection.csv" | head -1) $out/pmc_write/run_counter_collection.csv
mv $(find $out/p1 -name "*counter_collection.csv" | head -1) $out/pmc_valu/run_counter_collection.csv
python3 tools/traffic_summary.py $out $out > $out/traffic.txt
rm -f $out/trace/run_kernel_trace.csv $out/pmc_fetch/*.csv $out/pmc_write/*.csv $out/pmc_valu/*.csv
rm -rf $out/p1 $out/p2 $out/p3 $out/p4
cat $out/summary.txt
