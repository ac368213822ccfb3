#!/bin/bash
# round 3 check: changed GPU tests, smoke, the default bench line and the slab line at world 1
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_cv.py tests/test_gpu_slab.py \
  tests/test_gpu_cxx_mbs.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 python bench.py --mode slab --no-cpu > $O/slab1.json 2> $O/slab1.err && \
timeout -k 10 300 python bench.py --mode cv --steps 40 --warmup 5 > $O/cv4.json 2> $O/cv4.err && \
timeout -k 10 300 python bench.py --mode cv --steps 40 --warmup 5 --cv-batch 1 > $O/cv1.json 2> $O/cv1.err
