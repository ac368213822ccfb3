#!/bin/bash
# fused 3-D kernel: dim-2 chunking sweep (probe build in multivartv_amd/lib_p) at 256^3, 512^3, 512x512x64
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3b
mkdir -p $O
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_p/libmvtv.so
timeout -k 10 200 python tools/zchunk_probe.py 256 3952 1976 1520 1216 988 760 608 > $O/z256.txt 2>&1 && \
timeout -k 10 300 python tools/zchunk_probe.py 512 4736 2368 3848 7696 9472 1184 > $O/z512.txt 2>&1 && \
timeout -k 10 200 python tools/zchunk_probe.py 512x512x64 3848 2368 1184 592 > $O/z512x64.txt 2>&1 && \
for v in 16 32 16 32; do
  MVTV_TRI_TQ=$v timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --steps 30 --warmup 3 > $O/tri_tq$v.json 2> $O/tri_tq$v.err || exit 1
  python -c "import json;d=json.load(open('$O/tri_tq$v.json'));print('tq $v', d['ms_per_step'], d['kernels']['dct'], d['kernels']['dct_first'])" >> $O/tri.txt
done
unset MVTV_LIB_PATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_slab.py > $O/slab_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --mode cv --steps 40 --warmup 5 > $O/cv4.json 2> $O/cv4.err && \
timeout -k 10 300 python bench.py --mode cv --steps 40 --warmup 5 --cv-batch 2 > $O/cv2.json 2> $O/cv2.err
