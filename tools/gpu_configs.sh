#!/bin/bash
# one bench line per BASELINE config (with cpu_baseline), then a kernel trace of each shorter run
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/${CFG_OUT:-gpurun_out/cfg}
mkdir -p $O
cd $R
if [ -n "$CFG_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread $CFG_TESTS > $O/tests.log 2>&1 || exit 1
fi
run() {  # name, args...
  local n=$1; shift
  echo "== $n $*" >> $O/progress.log
  timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err
}
run b512 && run b1024 --dims 2 --size 1024 && run b2048 --dims 2 --size 2048 && run b256 --dims 3 --size 256 && \
run b128_4d --dims 4 --size 128 --pcg-steps 4 && run bcv --mode cv --steps 40 --warmup 5 && \
run bslab1 --mode slab --no-cpu && \
run b500 --dims 3 --size 500 --steps 10 --warmup 2 --pcg-steps 5 && run b1000 --dims 2 --size 1000 --pcg-steps 20 && \
run b251 --dims 3 --size 251 --pcg-steps 10 && run b1009 --dims 2 --size 1009 --pcg-steps 20 || exit 1
cd /tmp && export TMPDIR=/tmp
kt() {
  local n=$1; shift
  echo "== kt $n $*" >> $O/progress.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@" > $O/kt_$n.log 2>&1
}
kt b1024 --dims 2 --size 1024 --pcg-steps 2 && kt bcv --mode cv --steps 20 --warmup 2 --cv-batch 1 && \
kt b128_4d --dims 4 --size 128 --steps 5 --warmup 2 --pcg-steps 0 && kt b256 --dims 3 --size 256 --pcg-steps 0
echo "rc=$?"
