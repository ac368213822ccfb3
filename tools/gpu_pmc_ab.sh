# GPU box: FETCH_SIZE / WRITE_SIZE of the short bench under each environment of AB_ENVS
# (one rocprofv3 --pmc pass per counter per environment), then the timing A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcab
cd /tmp && export TMPDIR=/tmp
for e in base $AB_ENVS; do
  if [ "$e" = base ]; then ev=""; else ev="$e"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    env $ev timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmcab/$e.$c -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 2 --warmup 1 > $R/gpurun_out/pmcab/$e.$c.log 2>&1 || { echo "pmc $e $c failed"; tail -5 $R/gpurun_out/pmcab/$e.$c.log; exit 1; }
  done
done
cd $R && bash tools/gpu_ab_env.sh
