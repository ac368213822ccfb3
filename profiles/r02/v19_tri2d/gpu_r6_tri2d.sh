#!/bin/bash
# 2-D last-dimension pass by the tridiagonal solve: spectral / config tests (release library), then a
# same-box A/B against the FFT pass (probe library, MVTV_DCT_TRI2D=0) and 8-line tiles (=8)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/t2d
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
one() {  # tag env args...
  local t=$1 e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 "$@" > $O/$t.json 2> $O/$t.err || { tail -5 $O/$t.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels'].items()})" $O/$t.json $t
}
A1="--dims 2 --size 1024 --steps 300"
A2="--dims 2 --size 2048 --steps 200"
for rep in 1 2; do
  one k1_tri4.$rep X=1 $A1 && one k1_fft.$rep MVTV_DCT_TRI2D=0 $A1 && one k1_tri8.$rep MVTV_DCT_TRI2D=8 $A1 && \
  one k2_tri4.$rep X=1 $A2 && one k2_fft.$rep MVTV_DCT_TRI2D=0 $A2 && one k2_tri8.$rep MVTV_DCT_TRI2D=8 $A2 && \
  one cv_tri4.$rep X=1 --mode cv --steps 40 --warmup 5 && one cv_fft.$rep MVTV_DCT_TRI2D=0 --mode cv --steps 40 --warmup 5 || exit 1
done
echo "rc=$?"
