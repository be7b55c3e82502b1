mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/par.log 2>&1 || { tail -30 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --batch 8192 --no-cpu-baseline > gpurun_out/exp.log 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads(open('gpurun_out/exp.log').read().strip().splitlines()[-1]); print(d['value'], {k: round(v/4,2) for k,v in d['kernels_ms_total'].items()})"
