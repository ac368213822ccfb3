# round 5: the mixed-radix / prime-length passes of the R API's default meshes —
#  (l) k_trig (the last-dimension line solves) on k_tris's wide tiles, and for prime lengths with a shorter last
#      segment (251^3: instead of the Bluestein MID pass); MVTV_TRIG_NARROW=1 MVTV_TRIG_EXACT=1: round 4's form;
#  (m) strided passes with their tiles dealt to the XCDs in contiguous runs (xcd_run: a 4000-B / 2008-B / 800-B line
#      pitch puts a tile's 128-B row across two lines, which round-robin dealing fetched through two L2s);
#      MVTV_XRUN_OFF=1: round-robin.
# Spectral / fused / config tests on the release build, then the two A/Bs on the probe build, interleaved, then kernel
# traces of 500^3 and 251^3 on the release build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5l
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_spectral.py tests/test_gpu_fused3d.py tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
run() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --size $N --steps 20 --warmup 3 --no-cpu --pcg-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2],d['value'],d['ms_per_step'],k['dct']['avg_ms'],k['dct_first']['avg_ms'])" $O/$tag.json "$tag"
}
for rep in 1 2; do
  for N in 500 251 100; do
    run l$N.old.$rep MVTV_TRIG_NARROW=1 MVTV_TRIG_EXACT=1 MVTV_XRUN_OFF=1 || exit 1
    run l$N.trig.$rep MVTV_XRUN_OFF=1 || exit 1
    run l$N.both.$rep MVTV_XRUN_OFF=0 || exit 1
  done
done
unset MVTV_LIB_PATH
cd /tmp && export TMPDIR=/tmp
for n in 500 251; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$n -o run --output-format csv -- python3 $R/bench.py --size $n --no-cpu --pcg-steps 0 --steps 10 --warmup 2 > $O/kt$n.log 2>&1 || { echo "trace $n failed"; exit 1; }
done
echo done
