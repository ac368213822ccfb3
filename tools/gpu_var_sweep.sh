# Compare fused-PCG variants (MVTV_CG3D_VAR) at 512^3; parity of variant ${CHECK_VAR:-3} first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MVTV_CG3D_VAR=${CHECK_VAR:-3} timeout -k 10 400 python -m pytest tests/test_gpu_cg3d.py -q -m gpu -x > gpurun_out/var_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/var_tests.log; exit 1; }
for v in ${VARS:-0 1 2 3}; do
  MVTV_CG3D_VAR=$v timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/var$v.json 2> gpurun_out/var$v.err || { echo "bench var $v failed"; exit 1; }
  echo "var $v"; cat gpurun_out/var$v.json
done
