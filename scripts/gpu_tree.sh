# Tree kernel bring-up: its parity tests, then the configs[3] (MPC) bench leg.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py -k "tree" -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_tree.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_tree.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tree_bench.py $TREE_CASES > gpurun_out/tree_bench.log 2>&1; rc=$?; echo "tree bench rc=$rc"; cat gpurun_out/tree_bench.log | tail -20
