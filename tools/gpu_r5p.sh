# round 5: k_trig's segment length at 500^3 — 20 rows (25 segments: 32-line tiles, the default), 32 rows with a
# 20-row last segment (16 segments: 64-line tiles, one 512-B row a wave load), 16 rows with a 4-row last one (32
# segments, 32-line tiles, 16 row registers). Probe build, interleaved, then a trace of each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5p
mkdir -p $O
cd $R
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
timeout -k 10 600 env MVTV_TRIG_SL=32 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_spectral.py -k "residual" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
run() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --size 500 --steps 20 --warmup 3 --no-cpu --pcg-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2],d['value'],d['ms_per_step'],k['dct']['avg_ms'],k['dct_first']['avg_ms'])" $O/$tag.json "$tag"
}
for rep in 1 2; do
  run sl20.$rep MVTV_TRIG_SL=20 || exit 1
  run sl32.$rep MVTV_TRIG_SL=32 || exit 1
  run sl16.$rep MVTV_TRIG_SL=16 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for sl in 20 32 16; do
  MVTV_TRIG_SL=$sl timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_sl$sl -o run --output-format csv -- python3 $R/bench.py --size 500 --no-cpu --pcg-steps 0 --steps 5 --warmup 1 > $O/kt_sl$sl.log 2>&1 || { echo "trace failed"; exit 1; }
done
echo done
