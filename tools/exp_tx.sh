# TX section-skip experiment (DNRP_TX_DBG bit 1: no cell mapping, 2: no IFFT, 4: no resampler)
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for d in 0 1 2 4 7; do
  DNRP_TX_RUN=2 DNRP_TX_DBG=$d timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY \
     --output-format csv -d gpurun_out/exp/d$d -o run -- python3 bench.py --steps 1 --warmup 0 --batch 4096 --no-cpu-baseline > gpurun_out/exp/d$d.log 2>&1 || exit 1
  DNRP_TX_RUN=2 DNRP_TX_DBG=$d timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --batch 4096 --no-cpu-baseline > gpurun_out/exp/t$d.log 2>&1 || exit 1
  python3 - $d <<'PY'
import csv, json, sys, collections
d = sys.argv[1]
rows = [r for r in csv.DictReader(open(f"gpurun_out/exp/d{d}/run_counter_collection.csv")) if "tx_kernel" in r["Kernel_Name"]]
agg = collections.defaultdict(float)
for r in rows: agg[r["Counter_Name"]] += float(r["Counter_Value"])
w = agg["SQ_WAVES"]
t = json.loads(open(f"gpurun_out/exp/t{d}.log").read().strip().splitlines()[-1])["kernels_ms_total"]["tx"] / 2
print(d, f"tx {t:.2f} ms", {k: round(v / w) for k, v in agg.items() if k != "SQ_WAVES"}, int(w))
PY
done
rm -rf gpurun_out/exp/d*
