# round 5: tiles of the mixed-radix passes for few lines (2-D meshes: 1000 x 1000 has 1000 lines a pass, 63 tiles of
# 16) — k_dctg / k_dctm tiles halved until the grid has >= 512 workgroups; k_dctm's 8-line tile at 1000 too.
# old = MVTV_FEW_LINES_OFF=1 MVTV_DCTM_NCL=8 (round 4's tiles), mid = MVTV_FEW_LINES_OFF=1 (8-line k_dctm only),
# new = the release build's choice. Tests on the release build, then the A/B on the probe build, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5o
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_spectral.py tests/test_gpu_fused3d.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
run() {   # tag dims size env...
  local tag=$1 dims=$2 size=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --dims $dims --size $size --steps 20 --warmup 3 --no-cpu --pcg-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2],d['value'],d['ms_per_step'],k['dct']['avg_ms'],k['dct_first']['avg_ms'])" $O/$tag.json "$tag"
}
for rep in 1 2; do
  for cfg in "2 1000" "2 500" "3 500"; do
    set -- $cfg
    run old.$1d$2.$rep $1 $2 MVTV_FEW_LINES_OFF=1 MVTV_DCTM_NCL=8 || exit 1
    run mid.$1d$2.$rep $1 $2 MVTV_FEW_LINES_OFF=1 || exit 1
    run new.$1d$2.$rep $1 $2 MVTV_FEW_LINES_OFF=0 || exit 1
  done
done
echo done
