#!/bin/bash
# round-5 NN changes (affine activations, cell, binary post, totals): suite; A/B vs round start;
# VAD with 7 LSTM waves (abtest/lw7, PIPE_LW_SMALL=7): its parity and A/B; S2I acc32 vs acc64
set -o pipefail
O=gpurun_out/r05/g8; mkdir -p $O
export TMPDIR=/tmp
bash profiles/r05/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so - abtest/lw7/nnsp_amd/libnnsp_mi355x.so" 3 || exit 1
python -c "import json; d=json.load(open('gpurun_out/r05/ab_NNSP_LIB/2_1.json')); print('host_gap_ms', d['cascade']['host_gap_ms'], 'chunk_device_ms', d['cascade']['chunk_device_ms'])"
for a in "" "--acc32"; do for i in 1 2; do timeout -k 10 300 python bench.py --net s2i --no-cpu-baseline $a > $O/s2i${a}_$i.json 2>> $O/s2i.err || { echo "s2i bench failed"; exit 1; }; python -c "import json; d=json.load(open('$O/s2i${a}_$i.json')); print('s2i $a', round(d['value']/1e9,4), round(d['nn_ms_per_step'],4))"; done; done
bash profiles/r05/ab.sh NNSP_NET_PRIO "- 5 7" 2 || exit 1
export NNSP_NET_PRIO=5
bash profiles/r05/ab.sh NNSP_R0_ORDER "3 4" 2 || exit 1
echo all-ok
