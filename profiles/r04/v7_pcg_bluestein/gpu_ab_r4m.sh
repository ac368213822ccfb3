#!/bin/bash
# same-box A/B: fused PCG with the every-other-iteration x update (lib) vs HEAD (lib_ab) at 512^3, and the
# register-stage Bluestein passes k_dctb8 vs the LDS-staged k_dctb (probe lib, MVTV_DCTB_LDS=1) at 251^3 / 1009^2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4m
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_spectral.py > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d.get('pcg_leg',{}).get('value'),d.get('pcg_leg',{}).get('kernel_avg_ms'),{k:v['avg_ms'] for k,v in d['kernels'].items()})" $1 $2; }
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then L=$R/multivartv_amd/lib_ab/libmvtv.so; else L=$R/multivartv_amd/lib/libmvtv.so; fi
    MVTV_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu > $O/b512_$v.$rep.json 2> $O/b512_$v.$rep.err || { tail -5 $O/b512_$v.$rep.err; exit 1; }
    summ $O/b512_$v.$rep.json b512_$v.$rep
  done
done
P=$R/multivartv_amd/lib_probe/libmvtv.so
for rep in 1 2; do
  for v in r8 lds; do
    if [ $v = lds ]; then export MVTV_DCTB_LDS=1; else unset MVTV_DCTB_LDS; fi
    MVTV_LIB_PATH=$P timeout -k 10 300 python bench.py --no-cpu --dims 3 --size 251 --pcg-steps 0 > $O/b251_$v.$rep.json 2> $O/b251_$v.$rep.err || { tail -5 $O/b251_$v.$rep.err; exit 1; }
    summ $O/b251_$v.$rep.json b251_$v.$rep
    MVTV_LIB_PATH=$P timeout -k 10 300 python bench.py --no-cpu --dims 2 --size 1009 --pcg-steps 0 > $O/b1009_$v.$rep.json 2> $O/b1009_$v.$rep.err || { tail -5 $O/b1009_$v.$rep.err; exit 1; }
    summ $O/b1009_$v.$rep.json b1009_$v.$rep
  done
done
echo rc=0
