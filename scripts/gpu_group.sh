# Plan-group check: group + trace GPU tests, the row-kernel parity tests, a short bench (no CPU leg).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_traces.py tests/test_gpu_parity.py tests/test_gpu_assemble.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_group.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_group.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --steps 100 --large-batch 0 > gpurun_out/bench_group.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_group.log | cut -c1-300; grep -o '"mixed_patterns": {.*}, "shapes"' gpurun_out/bench_group.log; grep -o '{"workload": "recorded.*' gpurun_out/bench_group.log
