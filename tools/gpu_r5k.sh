# round 5: critical-path collectives on the compute stream (lane 0; RCCL: a second communicator split off for the
# halos) — slab tests on the release build, then the G-rank share A/B on the probe build, interleaved: one lane
# (MVTV_SLAB_CRIT_SC=1, every collective on the collectives stream between hand-offs) against two
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5k
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_slab.py tests/test_gpu_slab_ipc.py tests/test_gpu_fullsize.py::test_metric_512_cubed_eight_rank_decomposition \
  tests/test_gpu_fullsize.py::test_config5_128_4d_eight_rank_decomposition > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so
for rep in 1 2; do
  for crit in 1 0; do
    for spec in "d3g2 512,512,256" "d3g8 512,512,64" "d4g8 128,128,128,16"; do
      set -- $spec
      tag=$1.sc$crit.$rep; mesh=$2
      MVTV_SLAB_CRIT_SC=$crit MVTV_SLAB_DISTRIBUTED=1 timeout -k 10 300 python bench.py --mode slab --mesh $mesh --steps 20 --warmup 3 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'])" $O/$tag.json "$tag $mesh"
    done
  done
done
