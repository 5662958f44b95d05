# Row-kernel experiment: phase timings + kernel times for two knob settings, then the row parity tests.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
A="${OPTS_A:-}"; B="${OPTS_B:-QPB_R_LATEFAC=0}"
for o in "$A" "$B"; do
  echo "== opts: $o"
  QPB_WAVE_OPTS="$o" timeout -k 10 120 python -u scripts/row_timing.py 1024 > gpurun_out/rx_t.log 2>&1 || { cat gpurun_out/rx_t.log | tail -5; exit 1; }
  grep "{" gpurun_out/rx_t.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['slowest'], sum(r['slowest'].values()))"
  QPB_WAVE_OPTS="$o" timeout -k 10 200 python -u scripts/tree_bench.py c1:wave:1024 c1:wave:1024 c1:wave:1048576 > gpurun_out/rx_b.log 2>&1 || { tail -5 gpurun_out/rx_b.log; exit 1; }
  grep "{" gpurun_out/rx_b.log | cut -c1-140
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q -k "wave or group" --timeout 120 --timeout-method thread > gpurun_out/rx_p.log 2>&1; rc=$?; tail -2 gpurun_out/rx_p.log; exit $rc
