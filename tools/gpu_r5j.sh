# round 5: the slab line solves (k_tris) on 64-line tiles with their LDS sized to the block — slab parity tests, then
# the per-rank share measurement of r5h again (G = 2 / 4 / 8 rank shares at world 1, distributed path)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5j
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_slab.py tests/test_gpu_slab_ipc.py tests/test_gpu_fullsize.py::test_metric_512_cubed_eight_rank_decomposition \
  tests/test_gpu_fullsize.py::test_config5_128_4d_eight_rank_decomposition > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
for spec in "d3g2 1 512,512,256" "d3g4 1 512,512,128" "d3g8 1 512,512,64" "d4g2 1 128,128,128,64" "d4g4 1 128,128,128,32" \
            "d4g8 1 128,128,128,16"; do
  set -- $spec
  tag=$1; dist=$2; mesh=$3
  MVTV_SLAB_DISTRIBUTED=$dist timeout -k 10 300 python bench.py --mode slab --mesh $mesh --steps 20 --warmup 3 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'])" $O/$tag.json "$tag $mesh dist=$dist"
done
cd /tmp && export TMPDIR=/tmp
MVTV_SLAB_DISTRIBUTED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g8_3d -o run --output-format csv -- python3 $R/bench.py --mode slab --mesh 512,512,64 --steps 20 --warmup 3 > $O/g8_3d.log 2>&1
echo "prof rc=$?"
