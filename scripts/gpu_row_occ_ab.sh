cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/occ.jsonl
for rep in 1 2; do for v in default 0 1024; do
  if [ $v = default ]; then unset QPB_ROW_OCC_BATCH; else export QPB_ROW_OCC_BATCH=$v; fi
  timeout -k 10 300 python -u bench.py --no-mixed --no-shapes --no-cpu > gpurun_out/occ_one.log 2>&1 || { tail -5 gpurun_out/occ_one.log; exit 1; }
  python3 -c "
import json,sys
r=[json.loads(l) for l in open('gpurun_out/occ_one.log') if l.startswith('{')][-1]
print(json.dumps({'occ': sys.argv[1], 'value': r['value'], 'kernel_ms': r['roofline']['kernel_ms'], 'kernel': r['roofline']['kernel'], 'large_ms': r['large_batch']['kernel_ms']}))" $v | tee -a gpurun_out/occ.jsonl
done; done
