#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
# Stops at the first step that faults / aborts / times out (rc 124,134,137,139).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$? ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$? ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$? ;;
    prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1; rc=$? ;;
    *) continue ;;
  esac
  echo "step $s rc=$rc"
  tail -3 gpurun_out/*.log 2>/dev/null | tail -0
  if fatal $rc; then echo "fatal rc=$rc at $s; stopping"; exit $rc; fi
done
exit 0
