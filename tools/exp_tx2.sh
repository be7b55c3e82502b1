mkdir -p gpurun_out/exp
for v in "DNRP_TX_STREAM=0" "DNRP_TX_STREAM=1"; do
  env $v timeout -k 10 200 python bench.py --steps 2 --warmup 1 --batch 4096 --no-cpu-baseline > gpurun_out/exp/s.log 2>&1 || { tail -5 gpurun_out/exp/s.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/exp/s.log').read().strip().splitlines()[-1]); print('$v', d['value'], round(d['kernels_ms_total']['tx']/2, 2), d['check']['pdc_hard_ber'])"
done
