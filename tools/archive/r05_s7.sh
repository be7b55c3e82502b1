#!/bin/bash
# Y residency probe: per-packet RX front-end / cells time vs device chunk (Y of a 64-packet chunk: 154 MB)
mkdir -p gpurun_out
for c in 32 64 128 512 4096; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --batch 4096 --chunk $c --no-cpu-baseline > gpurun_out/s7_$c.log 2>&1 || { tail -3 gpurun_out/s7_$c.log; exit 1; }
  tail -1 gpurun_out/s7_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_chunk']; c=$c; print(c, {n: round(v*1000/c,3) for n,v in k.items()}, 'us/packet')"
done
