# Cascade window sweep: frames/s, rounds per chunk and speculation overhead per window (0: whole chunk).
#   usage: profiles/sweep_window.sh [windows...]   (env passes through, e.g. NNSP_CASCADE_CONTROL_KERNEL=1)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for w in ${@:-4 8 12 16 24 32 0}; do
  timeout -k 10 120 python bench.py --window $w --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/sw_$w.json 2> gpurun_out/sw_$w.err || { tail -5 gpurun_out/sw_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw_$w.json'));print('w=$w',round(d['value']/1e6,2),'Mfr/s',d['cascade'], round(d['ms_per_step'],2))"
done
