# Parity tests + smoke + bench + drop-in latency (one GPU call).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; fatal $rc smoke
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.log; fatal $rc bench
: > gpurun_out/dropin_latency.jsonl
for sh in c1 c30 c30_trot c30_crawl; do for md in fast exact; do
  [ "$sh" != c1 ] && [ "$md" = exact ] && continue
  timeout -k 10 120 python -u scripts/dropin_latency.py --shape $sh --mode $md >> gpurun_out/dropin_latency.jsonl 2>gpurun_out/dl.err; rc=$?; echo "dropin $sh $md rc=$rc"; fatal $rc dropin
done; done
cut -c1-300 gpurun_out/dropin_latency.jsonl
