# GPU box, one parameterised A/B run (replaces round 5's one-off gpu_r5*.sh):
#   LIB=probe|release      library the steps load (probe: multivartv_amd/lib_probe, reads the MVTV_* knobs)
#   TESTS="tests/..."      pytest selection, run once per TEST_ENVS entry (";"-separated env sets, "" = none)
#   SWEEP="base;A=1 B=2"   env cases for the benches ("base" = no env), interleaved REPS times
#   CASES="3:512 4:128"    meshes (dims:size) per case; BENCH_EXTRA appended to every bench
#   KT=1                   each bench under rocprofv3 --kernel-trace, summarised per kernel (tools/prof_summary.py)
# Output: gpurun_out/$OUT/. Every GPU step is time-limited and the script stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-sweep}
mkdir -p $O
cd $R
if [ "${LIB:-probe}" = probe ]; then export MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so; fi
if [ -n "$TESTS" ]; then
  IFS=';' read -ra TE <<< "${TEST_ENVS:-}"
  [ ${#TE[@]} -eq 0 ] && TE=("")
  i=0
  for te in "${TE[@]}"; do
    i=$((i+1))
    env $te timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu $TESTS > $O/tests$i.log 2>&1
    rc=$?; echo "tests [$te]: $(tail -1 $O/tests$i.log)"
    if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
  done
fi
[ -z "$SWEEP" ] && exit 0
IFS=';' read -ra SW <<< "$SWEEP"
cd /tmp && export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  j=0
  for e in "${SW[@]}"; do
    j=$((j+1))
    if [ "$e" = base ]; then ev=""; else ev="$e"; fi
    for c in ${CASES:-3:512}; do
      d=${c%%:*}; n=${c##*:}
      f=$O/c$j.$d.$n.$rep
      echo "$e" > $f.case
      if [ "${KT:-0}" = 1 ]; then
        env $ev timeout -k 10 300 rocprofv3 --kernel-trace -d $f.kt -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps ${PCG_STEPS:-0} --steps ${STEPS:-20} --warmup 3 --dims $d --size $n ${BENCH_EXTRA} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
        python3 $R/tools/prof_summary.py $f.kt $f.kt.md > /dev/null
      else
        env $ev timeout -k 10 300 python3 $R/bench.py --no-cpu --pcg-steps ${PCG_STEPS:-0} --steps ${STEPS:-20} --warmup 3 --dims $d --size $n ${BENCH_EXTRA} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
      fi
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d.get('kernels',{});print(sys.argv[2],d['value'],d.get('pcg_leg',{}).get('value') if isinstance(d.get('pcg_leg'),dict) else '',json.dumps({a:round(b['avg_ms'],4) for a,b in k.items()}))" $f.json "[$e] $d:$n r$rep"
    done
  done
done
echo done
