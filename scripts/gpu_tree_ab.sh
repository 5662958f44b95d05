# Tree kernel A/B: parity tests on the default build, then MPC timings for the
# default and for each QPB_TREE_OPTS variant in $TREE_AB (';'-separated), interleaved.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_tree.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_tree.log
[ $rc -eq 0 ] || exit $rc
CASES=${TREE_CASES:-"mpc_h10:tree:1 mpc_h10:tree:512 mpc_h10:tree:1024"}
: > gpurun_out/tree_ab.log
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/tree_bench.py $CASES | sed "s/^/default /" >> gpurun_out/tree_ab.log; rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  IFS=';' read -ra VS <<< "${TREE_AB:-}"
  for v in "${VS[@]}"; do
    QPB_TREE_OPTS="$v" timeout -k 10 300 python -u scripts/tree_bench.py $CASES | sed "s/^/[$v] /" >> gpurun_out/tree_ab.log; rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  done
done
cat gpurun_out/tree_ab.log | cut -c1-220
