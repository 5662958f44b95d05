# Round-3 lazy pivot regularisation: GPU tests, then interleaved A/B of the row kernel
# (headline) and of the wave kernel (controller shapes + drop-in tick), off vs on.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PARTS=${PARTS:-test row wave tree}
if [[ $PARTS == *test* ]]; then bash scripts/gpu_pytest.sh || exit $?; fi
if [[ $PARTS == *row* ]]; then VARIANTS="QPB_R_LAZYREG=0;-" bash scripts/gpu_ab.sh || exit $?; fi
if [[ $PARTS == *wave* ]]; then
: > gpurun_out/lazy_dropin.jsonl
for rep in 1 2; do for v in "QPB_W_LAZYREG=0" "-"; do o="$v"; [ "$o" = "-" ] && o=""
  for sh in c1 c30; do
    QPB_WAVE_OPTS="$o" timeout -k 10 180 python -u scripts/dropin_latency.py --shape $sh --mode fast --ticks 300 > gpurun_out/dl_one.log 2>gpurun_out/dl.err || { echo "rc=$? $sh"; tail -5 gpurun_out/dl.err; exit 1; }
    python3 -c "import json,sys; r=json.loads(open('gpurun_out/dl_one.log').read().strip().splitlines()[-1]); r['variant']=sys.argv[1]; r['rep']=int(sys.argv[2]); print(json.dumps(r))" "$v" "$rep" | tee -a gpurun_out/lazy_dropin.jsonl | cut -c1-300
  done
  QPB_WAVE_OPTS="$o" timeout -k 10 300 python -u bench.py --no-mixed --no-cpu --steps 50 --large-batch 4096 > gpurun_out/lz_bench.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/lz_bench.log; exit 1; }
  python3 -c "
import json,sys
r=[json.loads(l) for l in open('gpurun_out/lz_bench.log') if l.startswith('{')][-1]
print(json.dumps({'variant': sys.argv[1], 'rep': int(sys.argv[2]), 'value': r['value'], 'shapes': r.get('shapes')}))" "$v" "$rep" | tee -a gpurun_out/lazy_dropin.jsonl | cut -c1-600
done; done
fi
if [[ $PARTS == *tree* ]]; then
: > gpurun_out/lazy_tree.log
for rep in 1 2; do for v in "QPB_T_LAZYREG=0" ""; do
  QPB_TREE_OPTS="$v" timeout -k 10 300 python -u scripts/tree_bench.py mpc_h10:tree:1024 mpc_h10:tree:1 | sed "s/^/[$v] /" >> gpurun_out/lazy_tree.log; rc=$?; [ $rc -eq 0 ] || exit $rc
done; done
cut -c1-220 gpurun_out/lazy_tree.log
fi
if [[ $PARTS == *timing* ]]; then
  for v in "" "QPB_R_LAZYREG=1"; do
    QPB_WAVE_OPTS="$v" timeout -k 10 200 python -u scripts/row_timing.py 1024 | sed "s/^/[$v] /" | tee -a gpurun_out/lazy_timing.log || exit 1
  done
fi
