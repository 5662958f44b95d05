# Drop-in check: drop-in tests (zero-copy default), then per-tick latency zero-copy vs staged.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dropin_t.log 2>&1; rc=$?; tail -2 gpurun_out/dropin_t.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/dropin_lat.jsonl
for sh in c1 c30; do for md in fast exact; do
  [ "$sh" = c30 ] && [ "$md" = exact ] && continue
  timeout -k 10 120 python -u scripts/dropin_latency.py --shape $sh --mode $md >> gpurun_out/dropin_lat.jsonl 2>gpurun_out/dl.err || { tail -3 gpurun_out/dl.err; exit 1; }
  QPSWIFT_HIP_STAGED=1 timeout -k 10 120 python -u scripts/dropin_latency.py --shape $sh --mode $md | sed 's/^{/{"staged": true, /' >> gpurun_out/dropin_lat.jsonl 2>gpurun_out/dl.err || { tail -3 gpurun_out/dl.err; exit 1; }
done; done
cut -c1-220 gpurun_out/dropin_lat.jsonl
