mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/par.log 2>&1 || { tail -30 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
for k in 2 3; do
for d in 0 4; do
  DNRP_TX_RUN=$k DNRP_TX_DBG=$d timeout -k 10 200 python bench.py --steps 1 --warmup 1 --batch 8192 --no-cpu-baseline > gpurun_out/exp_$d.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/exp_$d.log').read().strip().splitlines()[-1]); print($k, $d, {k: round(v/2,2) for k,v in d['kernels_ms_total'].items()})"
done
done
