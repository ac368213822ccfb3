# round 5: the slab loop picks its z ping-pong pair by timed probes — slab tests (loopback, ipc processes, the 8-rank
# decompositions), then a same-box A/B against the previous build of the slab line at world 1 (RCCL, one rank)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_slab.py tests/test_gpu_slab_ipc.py tests/test_gpu_fullsize.py::test_metric_512_cubed_eight_rank_decomposition \
  tests/test_gpu_zpick.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then L=$R/multivartv_amd/lib_ab/libmvtv.so; else L=$R/multivartv_amd/lib/libmvtv.so; fi
    f=$O/ab.$v.$rep
    MVTV_LIB_PATH=$L timeout -k 10 200 python bench.py --mode slab --steps 20 --warmup 3 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels_rank0'].items()})" $f.json "$v $rep"
  done
done
