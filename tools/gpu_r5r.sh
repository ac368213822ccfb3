# round 5: the last-dimension line solve (k_trig) for the few lines of 2-D meshes (8- / 4-line tiles) instead of the
# Bluestein / mixed-radix MID pass (MVTV_TRIG_FEW_OFF=1 keeps the MID pass). Tests on the release build, then the A/B
# at 1009^2 / 1000^2 / 500^2 / 2048^2-shaped on the probe build, interleaved, and a trace of 1009^2.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5r
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_spectral.py tests/test_gpu_fused3d.py tests/test_gpu_configs.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
run() {   # tag dims size env...
  local tag=$1 dims=$2 size=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --dims $dims --size $size --steps 20 --warmup 3 --no-cpu --pcg-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2],d['value'],d['ms_per_step'],k['dct']['avg_ms'],k['dct_first']['avg_ms'])" $O/$tag.json "$tag"
}
for rep in 1 2; do
  for n in 1009 1000 500 2039; do
    run off.2d$n.$rep 2 $n MVTV_TRIG_FEW_OFF=1 || exit 1
    run on.2d$n.$rep 2 $n MVTV_TRIG_FEW_OFF=0 || exit 1
  done
done
unset MVTV_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt1009 -o run --output-format csv -- python3 $R/bench.py --dims 2 --size 1009 --no-cpu --pcg-steps 0 --steps 20 --warmup 3 > $O/kt1009.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
