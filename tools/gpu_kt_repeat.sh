# GPU box: the bench under rocprofv3 --kernel-trace, once per env case (SWEEP="A=1;A=0"), to see
# per-launch duration patterns (e.g. ping-pong parity) of the fused kernel; summaries via
# tools/kt_pattern.py gpurun_out/ktr
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ktr
IFS=';' read -ra CASES <<< "$SWEEP"
i=0
cd /tmp && export TMPDIR=/tmp
for c in "${CASES[@]}"; do
  i=$((i+1))
  mkdir -p $R/gpurun_out/ktr/$i
  echo "$c" > $R/gpurun_out/ktr/$i/case.txt
  export $c
  timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/ktr/$i/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps ${STEPS:-12} --warmup 2 ${BENCH_ARGS} > $R/gpurun_out/ktr/$i/bench.json 2> $R/gpurun_out/ktr/$i/bench.err || { echo "case $i failed"; exit 1; }
  for kv in $c; do unset ${kv%%=*}; done
done
