#!/bin/bash
# 4-D on the chunked edge layout: parity tests, then 128^4 A/B (probe build, MVTV_EAOS=0 = block-major)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_slab.py \
  > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "4d or 128" \
  > $O/tests_full.log 2>&1 || exit 1
for v in 1 0 1 0; do
  MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_p/libmvtv.so MVTV_EAOS=$v timeout -k 10 300 python bench.py --dims 4 --size 128 --no-cpu --pcg-steps 0 --steps 6 --warmup 2 > $O/b128_eaos$v.json 2> $O/b128_eaos$v.err || exit 1
  python -c "import json;d=json.load(open('$O/b128_eaos$v.json'));k=d['kernels'];print('eaos $v', d['value'], d['ms_per_step'], k.get('edge_update'), k.get('gather_Dt'), k.get('gather4_b'))" >> $O/ab.txt
done
