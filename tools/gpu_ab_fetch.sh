# GPU box: A/B of env settings (SWEEP="A=1;A=0"): per case a short bench (timing) and one FETCH_SIZE
# pass (kernel-trace beside --pmc only) into gpurun_out/ab/<i>/. Read with tools/ab_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ab
IFS=';' read -ra CASES <<< "$SWEEP"
i=0
for c in "${CASES[@]}"; do
  i=$((i+1))
  mkdir -p $R/gpurun_out/ab/$i
  echo "$c" > $R/gpurun_out/ab/$i/case.txt
  cd $R
  env $c timeout -k 10 120 python bench.py --no-cpu --pcg-steps 0 --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/ab/$i/bench.json 2> gpurun_out/ab/$i/bench.err || { echo "bench case $i failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/$i/bench.json')); print('$c', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  if [ -z "$NOPMC" ]; then
    cd /tmp && export TMPDIR=/tmp
    export $c
    timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/ab/$i/fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 2 --warmup 1 ${BENCH_ARGS} > $R/gpurun_out/ab/$i/fetch.log 2>&1 || { echo "pmc case $i failed"; exit 1; }
    for kv in $c; do unset ${kv%%=*}; done
  fi
done
