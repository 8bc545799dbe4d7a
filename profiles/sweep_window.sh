cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for w in 4 8 12 16 24 32 0; do
  timeout -k 10 120 python bench.py --window $w --no-cpu-baseline > gpurun_out/sw_$w.json 2> gpurun_out/sw_$w.err || { tail -5 gpurun_out/sw_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw_$w.json'));print('w=$w',round(d['value']/1e6,2),'Mfr/s',{k:round(v,2) for k,v in d['kernels_ms_per_step'].items()},d['cascade'], round(d['ms_per_step'],2))"
done
