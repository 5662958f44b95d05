# Round 4: the resident warm solve reading its state from a host-only block (KernelArgs::win):
# (1) multi-request waves with round 3's cold kernel (QPB_W_SIGOUT=0) and today's; (2) the
# drop-in / persistent-solver GPU tests in multi-request mode (QPSWIFT_HIP_SERVE_LIFE_MS=10,
# QPB_SERVE_DIAG=1) and in the shipped one-request mode.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
O=QPB_WAVE_OPTS=QPB_W_SIGOUT
bash scripts/gpu_serve_diag.sh winA_nosig:$O=0 winB_nosig:$O=0 winC || exit 1
for m in multi oneshot; do
  ( [ $m = multi ] && export QPSWIFT_HIP_SERVE_LIFE_MS=10 QPB_SERVE_DIAG=1
    timeout -k 10 600 python -u -m pytest tests/test_serve.py tests/test_dropin.py tests/test_c_caller.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -k "not config3 and not config4" > gpurun_out/pytest_$m.log 2>&1; rc=$?
    echo "pytest [$m] rc=$rc $(tail -1 gpurun_out/pytest_$m.log)"; grep -E "^FAILED" gpurun_out/pytest_$m.log | head; fatal $rc pytest_$m; exit 0 ) || exit 1
done
