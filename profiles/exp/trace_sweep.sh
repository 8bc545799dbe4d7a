# cascade kernel trace (one rocprofv3 run) + a window sweep
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/ts
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ts/kt -o kt -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ts/kt.json 2> gpurun_out/ts/kt.err || { echo kt failed; tail -5 gpurun_out/ts/kt.err; exit 1; }
bash profiles/sweep_window.sh ${@:-10 12 14 16}
