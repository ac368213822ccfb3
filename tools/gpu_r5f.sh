# round 5: wave-only exchange sync in the d = 0 DCT passes — spectral / fused / parity tests on the new build, then
# a same-box interleaved A/B against the previous build (lib_ab) at 512^3, 256^3 and 1024^2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5f
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_spectral.py tests/test_gpu_fused3d.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py::test_metric_config_512_cubed \
  tests/test_gpu_fullsize.py::test_metric_config_512_cubed_vs_c_oracle tests/test_gpu_fullsize.py::test_config5_4d_128_single_gpu tests/test_gpu_fullsize.py::test_config5_128_4d_vs_c_oracle tests/test_gpu_cv.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
for rep in 1 2 3; do
  for v in new old; do
    for c in 3:512 3:256 2:1024 4:128; do
      d=${c%%:*}; n=${c##*:}
      if [ $v = old ]; then L=$R/multivartv_amd/lib_ab/libmvtv.so; else L=$R/multivartv_amd/lib/libmvtv.so; fi
      f=$O/ab.$v.$d.$n.$rep
      MVTV_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --dims $d --size $n > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels'].items()})" $f.json "$v $d:$n $rep"
    done
  done
done
