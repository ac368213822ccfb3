#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/p7
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_spectral.py tests/test_gpu_parity.py tests/test_gpu_cv.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
one() {  # tag env args...
  local t=$1 e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --no-cpu "$@" > $O/$t.json 2> $O/$t.err || { tail -5 $O/$t.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['config'].get('pcg_iters_mean'),{k:v['avg_ms'] for k,v in d['kernels'].items()})" $O/$t.json $t
}
for rep in 1 2; do
  one cv_seven.$rep X=1 --mode cv --steps 40 --warmup 5 && one cv_nine.$rep MVTV_PCGS_NINE=1 --mode cv --steps 40 --warmup 5 && \
  one cv3_seven.$rep X=1 --mode cv --dims 3 --size 256 --steps 20 --warmup 3 && one cv3_nine.$rep MVTV_PCGS_NINE=1 --mode cv --dims 3 --size 256 --steps 20 --warmup 3 || exit 1
done
