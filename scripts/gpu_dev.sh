# Development check: all GPU tests, tree-kernel phase timings, kernel timings, a short bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_dev.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dev.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/tree_timing.py > gpurun_out/tree_timing.log 2>&1; rc=$?; echo "timing rc=$rc"; cat gpurun_out/tree_timing.log | grep case
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tree_bench.py $TREE_CASES > gpurun_out/tree_bench.log 2>&1; rc=$?; echo "tree bench rc=$rc"; grep case gpurun_out/tree_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --steps 100 > gpurun_out/bench_dev.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_dev.log | cut -c1-400
