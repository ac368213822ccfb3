# round 5: k_dct8's tiles at 512^3 (probe knobs of launch_dct8): 8-line tiles for the d = 0 / strided passes (half the
# LDS: four workgroups a CU instead of two), 32-line strided tiles (256-B rows), XCD runs. Probe build, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s
mkdir -p $O
cd $R
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
run() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --pcg-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2],d['value'],d['ms_per_step'],k['dct']['avg_ms'],k.get('dct_first_fold',k.get('dct_first'))['avg_ms'],k['admm_fused']['avg_ms'])" $O/$tag.json "$tag"
}
for rep in 1 2; do
  run base.$rep MVTV_DCT_T0=16 || exit 1
  run t0_8.$rep MVTV_DCT_T0=8 || exit 1
  run t1_8.$rep MVTV_DCT_T1=8 || exit 1
  run t01_8.$rep MVTV_DCT_T0=8 MVTV_DCT_T1=8 || exit 1
  run t1_32.$rep MVTV_DCT_T1=32 || exit 1
  run xcd.$rep MVTV_DCT_XCD=1 || exit 1
done
echo done
