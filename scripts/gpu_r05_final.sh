# Round 5 closing run on the final tree, in two gpurun calls (each within the 20-minute cap):
#   PART=1: GPU parity suite, smoke, bench (the driver's default command), the drop-in tick
#           per shape (scripts/dropin_latency.py)
#   PART=2: the rocprofv3 kernel trace of the same bench (per-kernel, per-grid durations),
#           one FETCH_SIZE and one WRITE_SIZE pass over a short bench (-> traffic.json), SQ
#           counter passes of the row kernel (headline) and of the band kernel (configs[3])
#   PART=3: SQ counter passes of the wave and wide-row kernels the bench names (gpu_sq_wave.sh)
#   PART=4: after a change that leaves the GPU suite green (run separately): bench, the
#           drop-in tick per shape and the rocprofv3 kernel trace of the bench
#   PART=5: the FETCH_SIZE / WRITE_SIZE passes (-> traffic.json) alone
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fin; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
if [ "${PART:-1}" = 1 ] || [ "${PART}" = 4 ]; then
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread > gpurun_out/fin/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/fin/pytest_gpu.log | head; tail -2 gpurun_out/fin/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/fin/smoke.log; fatal $rc smoke
fi
timeout -k 10 600 python bench.py > gpurun_out/fin/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/fin/bench.log; fatal $rc bench
: > gpurun_out/fin/dropin_latency.jsonl
for sh in c1 c30 c30_trot c30_crawl; do
  timeout -k 10 200 python -u scripts/dropin_latency.py --shape $sh --mode fast >> gpurun_out/fin/dropin_latency.jsonl 2>> gpurun_out/fin/dropin_latency.err; rc=$?
  echo "dropin latency $sh rc=$rc"; fatal $rc dropin_$sh
done
if [ "${PART}" = 4 ]; then
rm -rf gpurun_out/fin/prof; timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/fin/prof -o run -- python3 bench.py --no-cpu > gpurun_out/fin/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 scripts/prof_summary.py gpurun_out/fin/prof/run_results.db gpurun_out/fin/kernel_by_grid.csv gpurun_out/fin/kernel_stats.csv > /dev/null; echo "summary rc=$?"
fi
elif [ "${PART}" = 3 ]; then
bash scripts/gpu_sq_wave.sh > gpurun_out/fin/sq_wave.log 2>&1; rc=$?; echo "sq wave rc=$rc"; cat gpurun_out/fin/sq_wave.log | tail -6; fatal $rc sq_wave
cp gpurun_out/sqw/sq_wave.json gpurun_out/fin/sq_wave.json; cp gpurun_out/sqw/sq_rowx.json gpurun_out/fin/sq_rowx.json
else
if [ "${PART}" != 5 ]; then
rm -rf gpurun_out/fin/prof; timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/fin/prof -o run -- python3 bench.py --no-cpu > gpurun_out/fin/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 scripts/prof_summary.py gpurun_out/fin/prof/run_results.db gpurun_out/fin/kernel_by_grid.csv gpurun_out/fin/kernel_stats.csv > /dev/null; rc=$?; echo "summary rc=$rc"
fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/fin/pmc_$c -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/fin/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; fatal $rc pmc_$c; [ $rc = 0 ] || exit $rc
done
f=$(find gpurun_out/fin/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1); w=$(find gpurun_out/fin/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)
python3 scripts/traffic_all.py "$f" "$w" > gpurun_out/fin/traffic.log; echo "traffic rc=$?"; cp profiles/traffic.json gpurun_out/fin/traffic.json
[ "${PART}" = 5 ] && exit 0
SQDIR=gpurun_out/sq bash scripts/gpu_sq.sh > gpurun_out/fin/sq.log 2>&1; rc=$?; echo "sq rc=$rc"; fatal $rc sq
python3 scripts/sq_summary.py gpurun_out/sq gpurun_out/fin/sq_row.json > /dev/null; echo "sq summary rc=$?"
bash scripts/gpu_sq_band.sh > gpurun_out/fin/sq_band.log 2>&1; rc=$?; echo "sq band rc=$rc"; fatal $rc sq_band
python3 scripts/sq_summary.py gpurun_out/sqb gpurun_out/fin/sq_band.json band > /dev/null; echo "sq band summary rc=$?"
fi
