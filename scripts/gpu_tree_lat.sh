# Tree-kernel latency vs batch (MPC, configs[3]) at the default and 128-thread workgroups.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="mpc_h10:own:1:1e-6:tree mpc_h10:own:256:1e-6:tree mpc_h10:own:512:1e-6:tree mpc_h10:own:1024:1e-6:tree mpc_h10:own:2048:1e-6:tree"
: > gpurun_out/tl.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tl_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tl_pytest.log; [ $rc -eq 0 ] || exit $rc
for wg in 256 128; do
  QPB_TREE_WG=$wg timeout -k 10 300 python -u scripts/lat_bench.py $C ${EXTRA:-} >> gpurun_out/tl.jsonl 2>gpurun_out/tl.err || { tail -5 gpurun_out/tl.err; exit 1; }
done
cat gpurun_out/tl.jsonl
