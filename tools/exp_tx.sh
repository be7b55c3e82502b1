# TX experiment: run length K (DNRP_TX_RUN) x section skips (DNRP_TX_DBG bit 1: no cell mapping,
# 2: no IFFT, 4: no resampler) -> TX kernel ms per 4096-slot launch
mkdir -p gpurun_out/exp
for k in ${TX_KS:-2}; do
  for d in ${TX_DBGS:-0 7}; do
    DNRP_TX_RUN=$k DNRP_TX_DBG=$d timeout -k 10 200 python bench.py --steps 2 --warmup 1 --batch 4096 --no-cpu-baseline > gpurun_out/exp/k${k}d$d.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/exp/k${k}d$d.log').read().strip().splitlines()[-1]); print('K=$k dbg=$d tx ms', round(d['kernels_ms_total']['tx']/2, 2))"
  done
done
