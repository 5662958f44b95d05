# Round 6 GPU runs (one gpurun call per PART, each within the 20-minute cap):
#   PART=1: the GPU parity suite (the 17/20/6 wide-row case runs once in it), smoke, the
#           default bench; the kernels compiled on the box are copied back (kcache_box)
#   PART=2: rocprofv3 kernel trace of the bench + FETCH_SIZE / WRITE_SIZE passes
#   PART=3: SQ counter passes (row, wide row, band, wave kernels)
#   PART=4: bench + drop-in tick latency per shape
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
keep_cache() { rm -rf gpurun_out/r6/kcache_box; cp -r apf_quadruped_amd/kcache gpurun_out/r6/kcache_box; }
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r6/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r6/pytest_gpu.log | head -20; tail -2 gpurun_out/r6/pytest_gpu.log; keep_cache; fatal $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r6/smoke.log; keep_cache; fatal $rc smoke
  timeout -k 10 600 python bench.py > gpurun_out/r6/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r6/bench.log; keep_cache; fatal $rc bench
elif [ "${PART}" = 2 ]; then
  rm -rf gpurun_out/r6/prof; timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof -o run -- python3 bench.py --no-cpu > gpurun_out/r6/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
  python3 scripts/prof_summary.py gpurun_out/r6/prof/run_results.db gpurun_out/r6/kernel_by_grid.csv gpurun_out/r6/kernel_stats.csv > /dev/null; echo "summary rc=$?"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r6/pmc_$c -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r6/pmc_$c.log 2>&1
    rc=$?; echo "pmc $c rc=$rc"; fatal $rc pmc_$c; [ $rc = 0 ] || exit $rc
  done
  f=$(find gpurun_out/r6/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1); w=$(find gpurun_out/r6/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)
  python3 scripts/traffic_all.py "$f" "$w" > gpurun_out/r6/traffic.log; echo "traffic rc=$?"; cp profiles/traffic.json gpurun_out/r6/traffic.json
elif [ "${PART}" = 3 ]; then
  SQDIR=gpurun_out/sq bash scripts/gpu_sq.sh > gpurun_out/r6/sq.log 2>&1; rc=$?; echo "sq rc=$rc"; fatal $rc sq
  python3 scripts/sq_summary.py gpurun_out/sq gpurun_out/r6/sq_row.json > /dev/null; echo "sq summary rc=$?"
  bash scripts/gpu_sq_band.sh > gpurun_out/r6/sq_band.log 2>&1; rc=$?; echo "sq band rc=$rc"; fatal $rc sq_band
  python3 scripts/sq_summary.py gpurun_out/sqb gpurun_out/r6/sq_band.json band > /dev/null; echo "sq band summary rc=$?"
  bash scripts/gpu_sq_wave.sh > gpurun_out/r6/sq_wave.log 2>&1; rc=$?; echo "sq wave rc=$rc"; fatal $rc sq_wave
  cp gpurun_out/sqw/sq_wave.json gpurun_out/r6/sq_wave.json; cp gpurun_out/sqw/sq_rowx.json gpurun_out/r6/sq_rowx.json
elif [ "${PART}" = 4 ]; then
  timeout -k 10 600 python bench.py > gpurun_out/r6/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r6/bench.log; fatal $rc bench
  : > gpurun_out/r6/dropin_latency.jsonl
  for sh in c1 c30 c30_trot c30_crawl; do
    timeout -k 10 200 python -u scripts/dropin_latency.py --shape $sh --mode fast >> gpurun_out/r6/dropin_latency.jsonl 2>> gpurun_out/r6/dropin_latency.err; rc=$?
    echo "dropin latency $sh rc=$rc"; fatal $rc dropin_$sh
  done
  keep_cache
fi
