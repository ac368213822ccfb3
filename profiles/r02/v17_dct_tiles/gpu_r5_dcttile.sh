#!/bin/bash
# 2-D DCT tile sweep (probe library): d = 0 tile (MVTV_DCT_T0), strided tile (MVTV_DCT_T1), XCD runs
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dt
mkdir -p $O
cd $R
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
MVTV_DCT_T0=2 MVTV_DCT_T1=4 MVTV_DCT_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_configs.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
one() {  # tag env args...
  local t=$1 e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 "$@" > $O/$t.json 2> $O/$t.err || { tail -5 $O/$t.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels'].items()})" $O/$t.json $t
}
A1="--dims 2 --size 1024 --steps 300"
A2="--dims 2 --size 2048 --steps 200"
for rep in 1 2; do
  one k1_base.$rep X=1 $A1 && one k1_t0_2.$rep MVTV_DCT_T0=2 $A1 && one k1_t0_4.$rep MVTV_DCT_T0=4 $A1 && \
  one k1_t1_4.$rep MVTV_DCT_T1=4 $A1 && one k1_t1_8.$rep MVTV_DCT_T1=8 $A1 && \
  one k1_t1_4x.$rep "MVTV_DCT_T1=4 MVTV_DCT_XCD=1" $A1 && one k1_t1_8x.$rep "MVTV_DCT_T1=8 MVTV_DCT_XCD=1" $A1 && \
  one k1_t1_16x.$rep "MVTV_DCT_XCD=1" $A1 && one k1_all.$rep "MVTV_DCT_T0=2 MVTV_DCT_T1=4 MVTV_DCT_XCD=1" $A1 && \
  one k2_base.$rep X=1 $A2 && one k2_t0_2.$rep MVTV_DCT_T0=2 $A2 && one k2_t1_4x.$rep "MVTV_DCT_T1=4 MVTV_DCT_XCD=1" $A2 && \
  one k2_t1_8x.$rep "MVTV_DCT_XCD=1" $A2 && one k2_t1_2x.$rep "MVTV_DCT_T1=2 MVTV_DCT_XCD=1" $A2 && \
  one k2_all.$rep "MVTV_DCT_T0=2 MVTV_DCT_T1=4 MVTV_DCT_XCD=1" $A2 || exit 1
done
echo "rc=$?"
