# Compare kernel configurations at 512^3: SWEEP is a list of env assignments, one bench each
# (e.g. SWEEP="MVTV_CG3D_NZ=1 MVTV_CG3D_NZ=2"). Optional CHECK=1 runs the fused-PCG tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$CHECK" ]; then
  timeout -k 10 400 python -m pytest tests/test_gpu_cg3d.py -q -m gpu -x > gpurun_out/var_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/var_tests.log; exit 1; }
fi
i=0
for v in ${SWEEP:-NONE=0}; do
  env $v timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-10} --warmup 3 > gpurun_out/sweep$i.json 2> gpurun_out/sweep$i.err || { echo "bench $v failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep$i.json')); k=d['kernels']; print('$v', d['value'], 'fused', k['pcg_fused3d']['avg_ms'], 'edge', k['edge_update']['avg_ms'], 'gather', k['gather_Dt']['avg_ms'], 'init', k['pcg_init']['avg_ms'])"
  i=$((i+1))
done
if [ -n "$FETCH" ]; then
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  rm -rf $R/gpurun_out/prof_fetch
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/prof_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 2 --warmup 1 > $R/gpurun_out/prof_fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
  echo "fetch pass done"
fi
