# GPU box: the default bench from the current tree and from ./_old (another commit, built in place),
# alternating, fused-kernel and DCT timings side by side on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/abold
for i in 1 2 3; do
  for t in cur old; do
    d=$R; [ $t = old ] && d=$R/_old
    cd $d && timeout -k 10 150 python bench.py --no-cpu --pcg-steps 0 --steps 10 --warmup 2 > $R/gpurun_out/abold/$t$i.json 2> $R/gpurun_out/abold/$t$i.err || exit 1
    python -c "import json; d=json.load(open('$R/gpurun_out/abold/$t$i.json')); print('$t', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  done
done
