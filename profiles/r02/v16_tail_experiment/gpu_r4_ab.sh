#!/bin/bash
# same-box A/B (probe library): in-kernel tails vs separate finalize/control launches (MVTV_TAIL=0),
# four-launch vs nine-launch spectral PCG (MVTV_PCGS_NINE=1); interleaved runs
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab4
mkdir -p $O
cd $R
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
one() {  # tag env args...
  local t=$1 e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --no-cpu "$@" > $O/$t.json 2> $O/$t.err || { tail -5 $O/$t.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels'].items()})" $O/$t.json $t
}
for rep in 1 2; do
  one b512_tail.$rep MVTV_X=1 --pcg-steps 0 --steps 30 && one b512_notail.$rep MVTV_TAIL=0 --pcg-steps 0 --steps 30 && \
  one b1024_tail.$rep MVTV_X=1 --dims 2 --size 1024 --pcg-steps 0 --steps 200 && one b1024_notail.$rep MVTV_TAIL=0 --dims 2 --size 1024 --pcg-steps 0 --steps 200 && \
  one cv3_four.$rep MVTV_X=1 --mode cv --dims 3 --size 256 --steps 20 --warmup 3 && one cv3_nine.$rep MVTV_PCGS_NINE=1 --mode cv --dims 3 --size 256 --steps 20 --warmup 3 || exit 1
done
echo "rc=$?"
