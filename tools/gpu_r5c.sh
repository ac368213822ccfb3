# round 5 probe A/B: streamed strided DCT passes (k_dct8s, MVTV_DCT_STREAM=1) — parity tests on the probe library
# with the switch on, then interleaved 512^3 / 256^3 / 128^4 bench runs without / with it
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c
mkdir -p $O
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_probe/libmvtv.so
MVTV_DCT_STREAM=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py::test_metric_config_512_cubed tests/test_gpu_spectral.py tests/test_gpu_fused3d.py \
  > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
for rep in 1 2; do
  for e in 0 1; do
    for c in 3:512 3:256 4:128; do
      d=${c%%:*}; n=${c##*:}
      f=$O/s$e.$d.$n.$rep
      if [ $e = 1 ]; then export MVTV_DCT_STREAM=1; else unset MVTV_DCT_STREAM; fi
      timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --steps 30 --warmup 5 --dims $d --size $n > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d.get('kernels',{}).items()})" $f.json "stream=$e $d:$n rep $rep"
    done
  done
done
