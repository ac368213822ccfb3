#!/bin/bash
# config 4 work items: PCG enqueue-ahead depth x concurrent items (probe build)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3d
mkdir -p $O
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_p/libmvtv.so
for b in 1 4; do
  for ah in -2 0 2 4; do
    MVTV_PCG_AHEAD=$ah timeout -k 10 200 python bench.py --mode cv --steps 40 --warmup 5 --cv-batch $b > $O/cv_b${b}_a${ah}.json 2> $O/cv_b${b}_a${ah}.err || exit 1
    python -c "import json;d=json.load(open('$O/cv_b${b}_a${ah}.json'));print('batch $b ahead $ah', d['value'], d['config']['pcg_iters_mean'], d['with_kernel_events']['ms_per_step'], d['ms_per_step'])" >> $O/summary.txt
  done
done
MVTV_PCG_AHEAD=0 timeout -k 10 200 python bench.py --mode cv --steps 40 --warmup 5 --cv-batch 8 > $O/cv_b8_a0.json 2> $O/cv_b8_a0.err && \
python -c "import json;d=json.load(open('$O/cv_b8_a0.json'));print('batch 8 ahead 0', d['value'], d['config']['pcg_iters_mean'])" >> $O/summary.txt
unset MVTV_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_slab8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode slab --slab-ranks 8 --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$O/kt_slab8.log 2>&1
echo "rc=$?"
