# GPU parity tests only (configs first); the log lands in gpurun_out/pytest_gpu.log.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -cE "PASSED" gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR|Timeout" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit $rc
