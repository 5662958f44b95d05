# A/B of kernel source knobs on the headline + 2^20 legs: each variant in its own
# process, interleaved (A B A B) so box-level drift hits both.  VARIANTS is a
# ';'-separated list of QPB_WAVE_OPTS strings ("-" = defaults; "env:VAR=V VAR2=V2" sets
# environment variables instead, e.g. "env:QPB_ROW_SPLIT=1").
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:--;QPB_DPP_NOP=0}"
: > gpurun_out/ab.jsonl
for rep in 1 2; do for v in "${VS[@]}"; do
  o="$v"; [ "$o" = "-" ] && o=""; ev=""
  case "$o" in env:*) ev="${o#env:}"; o="";; esac
  env $ev QPB_WAVE_OPTS="$o" timeout -k 10 300 python -u bench.py --no-mixed --no-shapes --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab_one.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "variant '$v' rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; }
  python3 -c "
import json,sys
r=[json.loads(l) for l in open('gpurun_out/ab_one.log') if l.startswith('{')][-1]
lb=r.get('large_batch') or {}
print(json.dumps({'variant': sys.argv[1], 'rep': int(sys.argv[2]), 'value': r['value'], 'kernel_ms': r['roofline']['kernel_ms'], 'large_kernel_ms': lb.get('kernel_ms'), 'large_value': lb.get('value')}))" "$v" "$rep" | tee -a gpurun_out/ab.jsonl
done; done
