# round 5: k_plane8 with the padded plane-image pitch — the plane / 4-D parity tests, a same-box A/B against the
# previous build at 128^4 (lib_ab), then the 128^4 kernel trace and FETCH_SIZE / WRITE_SIZE passes of the new build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5e
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py::test_config5_4d_128_single_gpu tests/test_gpu_fullsize.py::test_config5_128_4d_vs_c_oracle \
  tests/test_gpu_spectral.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then L=$R/multivartv_amd/lib_ab/libmvtv.so; else L=$R/multivartv_amd/lib/libmvtv.so; fi
    MVTV_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --dims 4 --size 128 --steps 10 --warmup 3 > $O/ab.$v.$rep.json 2> $O/ab.$v.$rep.err || { tail -5 $O/ab.$v.$rep.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels'].items()})" $O/ab.$v.$rep.json $v.$rep
  done
done
cd /tmp && export TMPDIR=/tmp
A="--no-cpu --pcg-steps 0 --dims 4 --size 128"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py $A --steps 5 --warmup 2 > $O/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o run --output-format csv -- python3 $R/bench.py $A --steps 2 --warmup 1 > $O/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o run --output-format csv -- python3 $R/bench.py $A --steps 2 --warmup 1 > $O/write.log 2>&1
echo "prof rc=$?"
