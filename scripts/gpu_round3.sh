# Round 3: parity tests (configs first) + smoke + bench + rocprof kernel stats (one GPU call).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
[ -e gpurun_out/FATAL ] && { echo "an earlier step of this call faulted: not starting"; exit 1; }
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | head -12; tail -15 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; fatal $rc smoke
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.log; fatal $rc bench
rm -rf gpurun_out/prof; timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 200 --no-cpu > gpurun_out/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 scripts/prof_summary.py gpurun_out/prof/run_results.db gpurun_out/kernel_by_grid.csv gpurun_out/kernel_stats.csv > /dev/null && head -8 gpurun_out/kernel_stats.csv
