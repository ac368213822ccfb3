# GPU box: UTCL1 translation hit/miss counters and UTCL2 busy per kernel over the short bench
# (one rocprofv3 --pmc pass per counter group), twice (two processes, two placements).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tlb
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --kernel-trace -d $R/gpurun_out/tlb/tcp$rep -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 4 --warmup 1 > $R/gpurun_out/tlb/tcp$rep.log 2>&1 || { echo "tcp pass failed"; tail -5 $R/gpurun_out/tlb/tcp$rep.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/tlb/grbm$rep -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 4 --warmup 1 > $R/gpurun_out/tlb/grbm$rep.log 2>&1 || { echo "grbm pass failed"; tail -5 $R/gpurun_out/tlb/grbm$rep.log; exit 1; }
done
echo done
