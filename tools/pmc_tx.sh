#!/bin/bash
# SQ counter passes over the TX kernel alone (tools/tx_time.py) for the DNRP_TX_MFMA A/B:
# gpurun_out/pmc_tx/<mode>_p<i>/  (each pass its own run, gfx950 counter-slot limits)
set -e
export TMPDIR=/tmp
out=gpurun_out/pmc_tx
mkdir -p $out
for mode in 0 1; do
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
             "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
             "SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM"; do
    i=$((i+1))
    DNRP_TX_MFMA=$mode timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out/m${mode}_p$i -o run -- python3 tools/tx_time.py C4 4096 1 > $out/m${mode}_p$i.log 2>&1
  done
done
