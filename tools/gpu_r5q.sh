# round 5: (a) Bluestein passes for few lines (2-D 1009^2 / 251^2: one line pair per k_dctb8 workgroup when the default
# tile leaves < 512 workgroups; MVTV_FEW_LINES_OFF=1 keeps the default tile); (b) k_trig at 500^3 on 16 ragged segments
# of 32 rows (64-line tiles) against 25 of 20 (MVTV_TRIG_SL=20). Tests on the release build, A/B on the probe build,
# interleaved, then a kernel trace of 500^3 and 1009^2 on the release build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5q
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_spectral.py tests/test_gpu_fused3d.py tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
run() {   # tag dims size env...
  local tag=$1 dims=$2 size=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --dims $dims --size $size --steps 20 --warmup 3 --no-cpu --pcg-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2],d['value'],d['ms_per_step'],k['dct']['avg_ms'],k['dct_first']['avg_ms'])" $O/$tag.json "$tag"
}
for rep in 1 2; do
  run old.2d1009.$rep 2 1009 MVTV_FEW_LINES_OFF=1 || exit 1
  run new.2d1009.$rep 2 1009 MVTV_FEW_LINES_OFF=0 || exit 1
  run old.2d251.$rep 2 251 MVTV_FEW_LINES_OFF=1 || exit 1
  run new.2d251.$rep 2 251 MVTV_FEW_LINES_OFF=0 || exit 1
  run sl20.3d500.$rep 3 500 MVTV_TRIG_SL=20 || exit 1
  run new.3d500.$rep 3 500 MVTV_FEW_LINES_OFF=0 || exit 1
done
unset MVTV_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt500 -o run --output-format csv -- python3 $R/bench.py --size 500 --no-cpu --pcg-steps 0 --steps 5 --warmup 1 > $O/kt500.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt1009 -o run --output-format csv -- python3 $R/bench.py --dims 2 --size 1009 --no-cpu --pcg-steps 0 --steps 20 --warmup 3 > $O/kt1009.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
