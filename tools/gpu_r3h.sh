# Round 3, folded right-hand side: the changed-path GPU tests, smoke, then the 512^3 and 256^3 bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3h
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_fused3d.py tests/test_gpu_parity.py tests/test_gpu_spectral.py > gpurun_out/r3h/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3h/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3h/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/r3h/b512.json 2> gpurun_out/r3h/b512.err || exit $?
timeout -k 10 300 python bench.py --no-cpu --steps 40 --warmup 5 --size 256 > gpurun_out/r3h/b256.json 2> gpurun_out/r3h/b256.err || exit $?
python - <<'PY'
import json
for f in ("b512", "b256"):
    d = json.load(open(f"gpurun_out/r3h/{f}.json"))
    k = d.get("kernels", {})
    print(f, d["value"], d["ms_per_step"], {n: round(v["avg_ms"], 4) for n, v in k.items()})
PY
