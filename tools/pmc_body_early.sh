# PMC of k_body over C5's first 512 merges (the early, bandwidth-heavy merges):
# where a wave's cycles go (parked on memory / issue-stalled / issuing), LDS work
set -e
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out/r4e
cd /tmp
EXPLORE_REPS=1 EXPLORE_MAX_STEPS=4 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d /tmp/pb1 -o run -- python3 $R/tools/explore_1g.py code1g > $R/gpurun_out/r4e/pb1.log 2>&1
python3 $R/tools/pmc_kernel_sum.py /tmp/pb1 "k_body<unsigned int, false, 1024, 16, false>" > $R/gpurun_out/r4e/pmc_body_early.txt
python3 $R/tools/pmc_kernel_sum.py /tmp/pb1 "k_body<unsigned int, false, 1024, 16, true>" >> $R/gpurun_out/r4e/pmc_body_early.txt
EXPLORE_REPS=1 EXPLORE_MAX_STEPS=4 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES --output-format csv -d /tmp/pb2 -o run -- python3 $R/tools/explore_1g.py code1g > $R/gpurun_out/r4e/pb2.log 2>&1
python3 $R/tools/pmc_kernel_sum.py /tmp/pb2 "k_body<unsigned int, false, 1024, 16, false>" >> $R/gpurun_out/r4e/pmc_body_early.txt
python3 $R/tools/pmc_kernel_sum.py /tmp/pb2 "k_body<unsigned int, false, 1024, 16, true>" >> $R/gpurun_out/r4e/pmc_body_early.txt
cat $R/gpurun_out/r4e/pmc_body_early.txt
