#!/bin/bash
# SQ counter breakdown per wave of every kernel of one bench chunk (batch 1024, 1 step), plus L2 hit /
# miss: the fused PDC receiver against the Y-path front end (DNRP_RX_FUSED=$1, default 1).
# Summary -> gpurun_out/pmc_fused$1/summary.txt
v=${1:-1}
out=gpurun_out/pmc_fused$v
mkdir -p $out
export TMPDIR=/tmp
export DNRP_RX_FUSED=$v
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --batch 1024 --no-cpu-baseline > $out/p$i.log 2>&1 || { tail -5 $out/p$i.log; exit 1; }
done
python3 tools/pmc_r02_summary.py $out > $out/summary.txt
rm -rf $out/p1 $out/p2 $out/p3
grep -E "rx_fused|rx_fft_wave|rx_cells" $out/summary.txt
