# round 5: the inter-process slab tests (verbose, progress to a file), the default bench, the 2-process slab line
# through bench.py's launcher on the one GPU, then probe A/B of the streamed theta-solve passes and z-chunked pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_slab_ipc.py -v -s -x --timeout 280 --timeout-method thread > $O/ipc.log 2>&1
rc=$?; tail -12 $O/ipc.log
if [ $rc -ne 0 ]; then echo "ipc tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --mode slab --steps 10 --warmup 2 > $O/bench_slab2.json 2> $O/bench_slab2.err
rc=$?; echo "slab2 rc=$rc"; tail -3 $O/bench_slab2.err
if [ $rc -gt 1 ]; then exit $rc; fi
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_probe/libmvtv.so
MVTV_DCT_STREAM=1 MVTV_TRI_STREAM=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py::test_metric_config_512_cubed tests/test_gpu_fullsize.py::test_config5_4d_128_single_gpu \
  tests/test_gpu_spectral.py tests/test_gpu_fused3d.py > $O/stream_tests.log 2>&1
rc=$?; tail -3 $O/stream_tests.log
if [ $rc -ne 0 ]; then echo "stream tests rc=$rc: stopping"; exit $rc; fi
for rep in 1 2; do
  for ev in BASE=1 MVTV_ZCHUNK=64 MVTV_DCT_STREAM=1 MVTV_TRI_STREAM=1 "MVTV_DCT_STREAM=1 MVTV_TRI_STREAM=1"; do
    tag=$(echo $ev | tr ' =' '__')
    f=$O/ab.$tag.$rep
    env $ev timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --steps 30 --warmup 5 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d.get('kernels',{}).items()})" $f.json "$tag rep $rep"
  done
done
