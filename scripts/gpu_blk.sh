# Blocked LDL' A/B: wave / drop-in parity tests, drop-in C30 latency and the bench
# controller legs with QPB_W_BLK on (default for ND > 32) and off.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_assemble.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/blk_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/blk_pytest.log; fatal $rc pytest
: > gpurun_out/blk_dropin.jsonl
for v in "-" "QPB_W_BLK=0" "QPB_W_BLK=0 QPB_W_H0RE=0"; do
  o="$v"; [ "$o" = "-" ] && o=""
  for sh in c30 c30_trot; do
    QPB_WAVE_OPTS="$o" timeout -k 10 200 python -u scripts/dropin_latency.py --shape $sh --mode fast > gpurun_out/blk_one.jsonl 2>gpurun_out/blk_dl.err; rc=$?
    echo "dropin '$v' $sh rc=$rc"; fatal $rc dropin
    python3 -c "import json,sys; r=json.loads(open('gpurun_out/blk_one.jsonl').read().strip().splitlines()[-1]); r['variant']=sys.argv[1]; print(json.dumps(r))" "$v" | tee -a gpurun_out/blk_dropin.jsonl
  done
  QPB_WAVE_OPTS="$o" timeout -k 10 400 python -u bench.py --no-mixed --no-cpu --steps 50 --warmup 5 > gpurun_out/blk_bench_$rep${o// /_}.log 2>&1; rc=$?; echo "bench '$v' rc=$rc"; fatal $rc bench
done
