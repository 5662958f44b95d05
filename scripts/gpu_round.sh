# Round deliverables: parity tests, smoke, bench, rocprof stats + HBM PMC passes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; fatal $rc smoke
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; fatal $rc bench
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --no-cpu > gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"; fatal $rc prof
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o b -- python3 bench.py --no-cpu --steps 20 --warmup 2 > gpurun_out/pmc_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"; fatal $rc fetch
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o b -- python3 bench.py --no-cpu --steps 20 --warmup 2 > gpurun_out/pmc_write.log 2>&1; rc=$?; echo "write rc=$rc"; fatal $rc write
: > gpurun_out/dropin_latency.jsonl
for sh in c1 c30 c30_trot c30_crawl; do for md in fast exact; do
  [ "$sh" != c1 ] && [ "$md" = exact ] && continue
  timeout -k 10 120 python -u scripts/dropin_latency.py --shape $sh --mode $md >> gpurun_out/dropin_latency.jsonl 2>gpurun_out/dl.err; rc=$?; echo "dropin $sh $md rc=$rc"; fatal $rc dropin
done; done
