#!/bin/bash
# copy the round-6 PMC summaries into profiles/r06 (C4 -> traffic.json / valu.json, others suffixed)
set -e
d=profiles/r06
mkdir -p $d
for tag in c4 ypath c4sm; do
  src=gpurun_out/prof_r06_$tag
  suf=""; [ $tag != c4 ] && suf="_$tag"
  cp $src/traffic.json $d/traffic$suf.json
  cp $src/valu.json $d/valu$suf.json
  cp $src/traffic.txt $d/traffic$suf.txt
  cp $src/summary.txt $d/pmc_sq_summary$suf.txt
  cp $(find $src/trace -name "*kernel_stats.csv" | head -1) $d/kernel_stats_profile_run$suf.csv
done
# slots per launch of each summary (bench.py _pmc_chunk)
cat > $d/pmc_meta.json <<'J'
{"traffic.json": 16384, "valu.json": 16384, "traffic_ypath.json": 16384, "valu_ypath.json": 16384,
 "traffic_c4sm.json": 8192, "valu_c4sm.json": 8192}
J
