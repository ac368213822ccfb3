#!/bin/bash
# slab tests incl. W != I (distributed PCG-spectral) and the distributed-at-one-rank RCCL path; slab bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_slab.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode slab --no-cpu > $O/slab_solo.json 2> $O/slab_solo.err && \
MVTV_SLAB_DISTRIBUTED=1 timeout -k 10 200 python bench.py --mode slab --no-cpu > $O/slab_dist1.json 2> $O/slab_dist1.err && \
MVTV_SLAB_DISTRIBUTED=1 timeout -k 10 200 python bench.py --mode slab --no-cpu --dims 4 --size 128 --steps 6 --warmup 2 > $O/slab4d_dist1.json 2> $O/slab4d_dist1.err
