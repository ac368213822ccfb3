# GPU box: bench under a list of env settings (SWEEP="A=1 B=2;A=2 B=3"), one short run each.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sweep
cd $R
i=0
IFS=';' read -ra CASES <<< "$SWEEP"
for c in "${CASES[@]}"; do
  i=$((i+1))
  env $c timeout -k 10 120 python bench.py --no-cpu --pcg-steps 0 --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/sweep/$i.json 2> gpurun_out/sweep/$i.err || { echo "case $i ($c) failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep/$i.json')); print('$c', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
