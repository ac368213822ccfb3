# round 5: diagnose the 4-process 128^4 / 2-process 512^3 ipc slab runs (transport trace to stderr)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5d
mkdir -p $O
MVTV_IPC_TRACE=1 timeout -k 10 400 python -u -m pytest "tests/test_gpu_slab_ipc.py::test_slab_processes_match_one_gpu[config5_128_4d_4proc]" -v -s -x --timeout 250 --timeout-method thread > $O/ipc128.log 2>&1
echo "128^4 rc=$?"; grep -c "ipc " $O/ipc128.log
