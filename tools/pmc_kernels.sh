# Per-kernel SQ counter breakdown of one bench step (batch 1024): wave cycles split into
# waiting / issue-stalled / active, instruction mix, LDS bank conflicts. Summary -> gpurun_out/pmc/summary.txt
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --batch 1024 --no-cpu-baseline > gpurun_out/pmc/p$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void dnrp::dev::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
out = []
for k, c in sorted(agg.items()):
    w = c.get("SQ_WAVES", 0) or 1
    out.append(k + "  " + " ".join(f"{n}={v / w:.0f}" for n, v in sorted(c.items()) if n != "SQ_WAVES") + f" waves={w:.0f}")
open("gpurun_out/pmc/summary.txt", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
rm -rf gpurun_out/pmc/p1 gpurun_out/pmc/p2
