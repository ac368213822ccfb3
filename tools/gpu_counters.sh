# GPU box: SQ/TCC counter passes for the bench's kernels (each pass its own rocprofv3 run with
# --kernel-trace only beside --pmc), plus the list of counters this GPU exposes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${CTR_OUT:-ctr}   # always under gpurun_out (merged back)
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1
ARGS="--no-cpu --steps 1 --warmup 1 ${PROF_ARGS}"
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM" \
            "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace -d $O/ctr$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/ctr$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "exit 0"
