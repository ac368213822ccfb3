# GPU box, end-of-milestone evidence: full GPU test suite (achieved parity errors logged), the stream ceiling, the
# default bench (with cpu_baseline), the N = 2 launcher path on the one GPU (independent fits + the slab line over
# the ipc transport), a rocprofv3 kernel-trace of the bench, FETCH_SIZE / WRITE_SIZE passes (separate runs) and the
# PMC calibration copies, then smoke(). Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=${REL_OUT:-gpurun_out/rel}
mkdir -p $R/$O
cd $R
# SKIP_TESTS=1: the evidence steps only
rc=0
if [ -z "$SKIP_TESTS" ]; then
  MVTV_PARITY_LOG=$R/$O/parity.jsonl timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -2 $O/gpu_tests.log
  if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 120 tools/bin/stream_bench > $O/stream.txt 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 --pcg-steps 0 > $O/bench_n2.json 2> $O/bench_n2.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_kt -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 10 --warmup 2 > $R/$O/prof_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/prof_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 2 --steps 2 --warmup 1 > $R/$O/prof_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/prof_write -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 2 --steps 2 --warmup 1 > $R/$O/prof_write.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/calib_fetch -o run --output-format csv -- $R/tools/bin/pmc_calib > $R/$O/calib_fetch.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/calib_write -o run --output-format csv -- $R/tools/bin/pmc_calib > $R/$O/calib_write.log 2>&1
rc2=$?; cd $R; [ $rc2 -eq 0 ] && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "tests rc=$rc release rc=$rc2 smoke rc=$?"
