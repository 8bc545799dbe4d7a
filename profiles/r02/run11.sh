#!/bin/bash
# small check, GPU suite, smoke, default bench, torchrun (1 rank, RCCL) bench
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUTD:-r02w}
mkdir -p $O
NNSP_CASCADE_DEBUG=1 timeout -k 10 120 python -u profiles/r02/bisect_casc.py > $O/small.log 2>&1 || { tail -5 $O/small.log; exit 3; }
tail -1 $O/small.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 6; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 4; }
tail -c 400 $O/bench_default.json
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --no-cpu-baseline > $O/bench_torchrun1.json 2> $O/bench_torchrun1.err || { tail -5 $O/bench_torchrun1.err; exit 5; }
tail -c 300 $O/bench_torchrun1.json
echo done
