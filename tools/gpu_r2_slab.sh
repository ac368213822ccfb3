#!/bin/bash
# slab loop in libmvtv: loopback / RCCL parity tests, then slab bench at world 1 (RCCL) beside the one-GPU bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/slab
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --mode slab --steps 20 --warmup 3 > $O/slab_w1_$i.json 2> $O/slab_w1.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --pcg-steps 0 --no-cpu > $O/single_$i.json 2> $O/single.err || exit 1
done
timeout -k 10 300 python bench.py --mode slab --slab-ranks 8 --steps 10 --warmup 2 > $O/slab_r8.json 2> $O/slab_r8.err
echo "rc=$?"
