# round 5: k_dct8's strided passes in XCD runs by default — GPU tests of the spectral / config / full-size / parity
# paths on the release build, then the configs' bench lines (512^3, 256^3, 1024^2, 128^4).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5t
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_spectral.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py tests/test_gpu_fused3d.py tests/test_gpu_parity.py tests/test_gpu_slab.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
for cfg in "3 512" "3 256" "2 1024" "4 128"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --dims $1 --size $2 --steps 20 --warmup 3 --no-cpu --pcg-steps 0 > $O/b$1d$2.json 2> $O/b$1d$2.err || { tail -5 $O/b$1d$2.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2],d['value'],d['ms_per_step'],json.dumps({n:v['avg_ms'] for n,v in k.items()}))" $O/b$1d$2.json "b$1d$2"
done
echo done
