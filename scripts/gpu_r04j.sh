# Round 4: wave kernel -- structural-zero skip in the LDL' (QPB_W_LSKIP) and branch-free
# H0 (QPB_W_H0BF).  GPU parity suite, phase timing, then interleaved A/B (old = both off)
# of the bench's shape legs and of the drop-in tick (C1 / C30 stance, fast mode).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/j; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/j/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/j/pytest_gpu.log)"; grep -E "^FAILED|^ERROR" gpurun_out/j/pytest_gpu.log | head; fatal $rc pytest; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u scripts/wave_timing.py c1:amd c30:amd c30 > gpurun_out/j/wave_timing.jsonl 2> gpurun_out/j/wave_timing.err; rc=$?; echo "timing rc=$rc"; fatal $rc timing
OLD="QPB_W_H0BF=0 QPB_W_LSKIP=0"
for rep in 1 2; do for v in old new; do
  o=""; [ $v = old ] && o="$OLD"
  QPB_WAVE_OPTS="$o" timeout -k 10 400 python -u bench.py --no-cpu --no-mixed --steps 50 --warmup 10 > gpurun_out/j/bench_$v$rep.log 2>&1; rc=$?; echo "bench $v$rep rc=$rc"; fatal $rc bench; [ $rc = 0 ] || exit $rc
  python3 -c "
import json,sys
r=[json.loads(l) for l in open('gpurun_out/j/bench_$v$rep.log') if l.startswith('{')][-1]
print('$v$rep', ' '.join('%s=%.4g' % (s['workload'][:24].replace(' ','_'), s['kernel_ms']) for s in r['shapes']))"
  for sh in c1 c30; do
    QPB_WAVE_OPTS="$o" timeout -k 10 200 python -u scripts/dropin_latency.py --shape $sh --mode fast > gpurun_out/j/lat_${v}${rep}_$sh.json 2>> gpurun_out/j/lat.err; rc=$?; fatal $rc lat; [ $rc = 0 ] || exit $rc
    python3 -c "
import json
r=[json.loads(l) for l in open('gpurun_out/j/lat_${v}${rep}_$sh.json') if l.startswith('{')][-1]
print('$v$rep $sh', {k: r[k] for k in r if 'median' in k or k in ('optimal',)})"
  done
done; done
