#!/bin/bash
# 4-D gather pass A tile rows 4 / 8 / 16 (probe build), 128^4, two rounds; 4-D parity first
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/g4
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_slab.py -x -q --timeout 250 --timeout-method thread -k "4d or 4_d or 128 or config5" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PL=$R/multivartv_amd/lib_probe/libmvtv.so
B="python bench.py --no-cpu --dims 4 --size 128 --steps 5 --warmup 1 --pcg-steps 0"
for i in 1 2; do for ty in 4 8 16; do
  MVTV_LIB_PATH=$PL MVTV_G4_TY=$ty timeout -k 10 300 $B > $O/ty${ty}_$i.json 2>> $O/err.log || exit 1
done; done
for f in ty4_1 ty8_1 ty16_1 ty4_2 ty8_2 ty16_2; do python3 -c "import json; d=json.load(open('$O/$f.json')); k=d['kernels']; print('$f', d['value'], d['ms_per_step'], {n:v['avg_ms'] for n,v in k.items() if n.startswith('gather')})"; done
