# Tree kernel check: GPU tree tests, MPC / C30 tree timings, segment breakdown.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tc_p.log 2>&1; rc=$?; tail -2 gpurun_out/tc_p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/tree_bench.py mpc_h10:tree:1 mpc_h10:tree:1024 mpc_h10:tree:8192 c30:tree:1024 > gpurun_out/tc_b.log 2>&1 || { tail -3 gpurun_out/tc_b.log; exit 1; }
grep "{" gpurun_out/tc_b.log | cut -c1-140
timeout -k 10 120 python -u scripts/tree_segments.py mpc_h10:1 > gpurun_out/seg.log 2>&1; rc=$?; grep "{" gpurun_out/seg.log; exit $rc
