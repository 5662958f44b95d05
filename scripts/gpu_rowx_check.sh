# wide row kernel: parity tests (rowx + the controller-shape tests of test_gpu_parity.py),
# per-phase / per-part cycles, HIP-event timings vs the one-QP-per-wavefront form
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; out=gpurun_out/rowx_check.jsonl; : > $out
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_rowx.py tests/test_gpu_parity.py \
    -m gpu -k "rowx or c30 or controller or two_rows or structure_knobs" > gpurun_out/rowx_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/rowx_pytest.log; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python -u scripts/rowx_timing.py 1 1024 >> $out 2>/dev/null || exit $?
timeout -k 10 200 python -u scripts/rowx_timing.py --parts 1 1024 >> $out 2>/dev/null || exit $?
timeout -k 10 300 python -u scripts/tree_bench.py ${CASES:-c30:wave:1024 c30:wave1:1024 c30:wave:8192 c30:wave1:8192 c30:wave:1 c30:wave1:1} >> $out 2>/dev/null || exit $?
cat $out
