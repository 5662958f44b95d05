cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p6.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/p6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tree_segments.py mpc_h10:1 mpc_h10:1024 > gpurun_out/tseg.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/tseg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tree_bench.py c1:wave:1024 c1:wave:1048576 c1:wave:1024 c1:wave:1048576 > gpurun_out/rb.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rb.log | cut -c1-160; exit $rc
