# run the bench with each prebuilt library variant gpurun_var_libdnrp_*.so (kernel-constant sweeps)
mkdir -p gpurun_out/exp
cp dect-nr-plus-sdr_amd/libdnrp.so /tmp/libdnrp_orig.so
for f in gpurun_var_libdnrp_*.so; do
  cp $f dect-nr-plus-sdr_amd/libdnrp.so
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --batch 4096 --no-cpu-baseline > gpurun_out/exp/v.log 2>&1 || { tail -5 gpurun_out/exp/v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/exp/v.log').read().strip().splitlines()[-1]); k=d['kernels_ms_total']; print('$f', d['value'], {n: round(v/2,2) for n,v in k.items()})"
done
cp /tmp/libdnrp_orig.so dect-nr-plus-sdr_amd/libdnrp.so
