"""Average PMC counters per libdnrp kernel from rocprofv3 --pmc CSV outputs (tools/profile_r01.sh)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
for f in sorted(glob.glob(f"{root}/pmc_*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "dnrp" not in k:
            continue
        k = k.split("(")[0].replace("void dnrp::dev::", "").replace("dnrp::dev::", "")
        agg[(k, r["Grid_Size"], r["LDS_Block_Size"], r["VGPR_Count"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(f.split("/")[-2], k, {c: f"{sum(x) / len(x):.4g}" for c, x in v.items()})
