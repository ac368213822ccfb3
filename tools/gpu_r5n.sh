# round 5: 500^3 mixed-radix passes — k_dctm on 8-line tiles (MVTV_DCTM_NCL=4: 32 KB of LDS, up to five workgroups a
# CU, against 16-line tiles at two) and k_trig's segment length (MVTV_TRIG_SL=25: 20 segments against 25 of 20 rows);
# probe build, interleaved, then a kernel trace of the NCL=4 form
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5n
mkdir -p $O
cd $R
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
timeout -k 10 600 env MVTV_DCTM_NCL=4 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_spectral.py -k "residual_baseline or superlu" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
run() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --size 500 --steps 20 --warmup 3 --no-cpu --pcg-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2],d['value'],d['ms_per_step'],k['dct']['avg_ms'],k['dct_first']['avg_ms'])" $O/$tag.json "$tag"
}
for rep in 1 2; do
  run base.$rep MVTV_DCTM_NCL=8 || exit 1
  run ncl4.$rep MVTV_DCTM_NCL=4 || exit 1
  run sl25.$rep MVTV_TRIG_SL=25 || exit 1
done
cd /tmp && export TMPDIR=/tmp
MVTV_DCTM_NCL=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt500 -o run --output-format csv -- python3 $R/bench.py --size 500 --no-cpu --pcg-steps 0 --steps 10 --warmup 2 > $O/kt500.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
