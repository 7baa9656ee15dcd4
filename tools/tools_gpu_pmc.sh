set -e
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
B="python -u bench.py --steps 1 --warmup 0 --pods 2000 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc/p1 -o p1 -- $B > gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmc/p2 -o p2 -- $B > gpurun_out/pmc/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/kt -o kt -- $B > gpurun_out/pmc/kt.log 2>&1
find gpurun_out/pmc -name "*.csv" | head -20
