# Row-kernel knob bisection: each variant in its own process; the first failure ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for o in "QPB_R_ZF128=0 QPB_R_AADPP=0 QPB_R_LATEFAC=0" "QPB_R_ZF128=1" "QPB_R_AADPP=1" "QPB_R_LATEFAC=1" "QPB_R_ZF128=1 QPB_R_AADPP=1 QPB_R_LATEFAC=1"; do
  echo "== $o"
  QPB_WAVE_OPTS="$o" timeout -k 10 90 python -u scripts/tree_bench.py c1:wave:1024 c1:wave:1024 c1:wave:65536 > gpurun_out/bis.log 2>&1
  rc=$?; grep "{" gpurun_out/bis.log | cut -c1-150; [ $rc -eq 0 ] || { echo "rc=$rc"; grep -m3 -E "Error|error|Kernel Name" gpurun_out/bis.log; exit $rc; }
  QPB_WAVE_OPTS="$o" timeout -k 10 90 python -u scripts/row_timing.py 1024 > gpurun_out/bist.log 2>&1
  rc=$?; grep "{" gpurun_out/bist.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['slowest'], sum(r['slowest'].values()))"; [ $rc -eq 0 ] || exit $rc
done
