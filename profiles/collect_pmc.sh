set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --steps 3 --warmup 1"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/kt -o kt -- $B > gpurun_out/pmc/kt.log 2>&1; echo kt=$?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc/p1 -o p1 -- $B > gpurun_out/pmc/p1.log 2>&1; echo p1=$?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/p2 -o p2 -- $B > gpurun_out/pmc/p2.log 2>&1; echo p2=$?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/p3 -o p3 -- $B > gpurun_out/pmc/p3.log 2>&1; echo p3=$?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM --output-format csv -d gpurun_out/pmc/p4 -o p4 -- $B > gpurun_out/pmc/p4.log 2>&1; echo p4=$?
ls -R gpurun_out/pmc | head -40
