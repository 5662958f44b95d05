# GPU parity tests + one bench line (the round's quick check).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu > gpurun_out/bench_quick.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_quick.log | tail -1 | cut -c1-400; exit $rc
