#!/bin/bash
# A/B of library builds (tools/build_variant.sh) on one box: per build one short bench (serial-step
# kernel ms per chunk) and one rocprofv3 LDS / VALU counter pass over a 4096-slot step.
#   tools/ab_lib_pmc.sh base var1 var2 ...   (base = dect-nr-plus-sdr_amd/libdnrp.so)
# AB_ARGS: extra bench.py arguments. Summary lines on stdout, raw data under gpurun_out/ab/.
export TMPDIR=/tmp
out=gpurun_out/ab
mkdir -p $out
CNT="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for v in "$@"; do
  if [ "$v" = base ]; then lib=$PWD/dect-nr-plus-sdr_amd/libdnrp.so; else lib=$PWD/dect-nr-plus-sdr_amd/libdnrp_$v.so; fi
  DNRP_LIB=$lib timeout -k 10 240 python bench.py --steps 2 --warmup 1 --batch 16384 --no-cpu-baseline $AB_ARGS > $out/$v.log 2>&1 || { echo "$v bench failed"; tail -5 $out/$v.log; exit 1; }
  python3 - "$v" "$out/$v.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], {k: round(v, 3) for k, v in d['kernel_ms_per_chunk'].items()}, 'ber', round(d['check']['pdc_hard_ber'], 6), flush=True)
PY
  if [ -z "$NO_PMC" ]; then
    DNRP_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc $CNT --output-format csv -d $out/pmc_$v -o run -- python3 bench.py --steps 1 --warmup 0 --batch 4096 --chunk 4096 --no-cpu-baseline $AB_ARGS > $out/pmc_$v.log 2>&1 || { echo "$v pmc failed"; tail -5 $out/pmc_$v.log; exit 1; }
    python3 - "$v" "$out/pmc_$v" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void dnrp::dev::", "").split("<")[0]
        if k.startswith("rx_fft_wave_ct") or k.startswith("tx_stream") or k.startswith("rx_cells") or k.startswith("sync_steps") or k.startswith("sync_fine"):
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items()):
    w = c.get("SQ_WAVES", 1) or 1
    lds = c.get("SQ_INSTS_LDS", 0) or 1
    print(f"  {sys.argv[1]} {k}: waves {w:.0f} lds/wave {c.get('SQ_INSTS_LDS',0)/w:.0f} conflict/wave {c.get('SQ_LDS_BANK_CONFLICT',0)/w:.0f} "
          f"conflict/lds {c.get('SQ_LDS_BANK_CONFLICT',0)/lds:.3f} valu/wave {c.get('SQ_INSTS_VALU',0)/w:.0f} "
          f"wait_lds/cyc {c.get('SQ_WAIT_INST_LDS',0)/max(1,c.get('SQ_WAVE_CYCLES',1)):.3f}", flush=True)
PY
    rm -rf $out/pmc_$v
  fi
done
