# Tick latency of multi-request resident waves with the kernel arguments opaque per
# request (QPB_W_SERVE_OPQ=1, QPSWIFT_HIP_SERVE_LIFE_MS=10): scripts/dropin_latency.py.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sd5; export TMPDIR=/tmp
export QPSWIFT_HIP_SERVE_LIFE_MS=10 QPB_WAVE_OPTS="QPB_W_SERVE_OPQ=1"
: > gpurun_out/sd5/lat.jsonl
for sh in c30 c30_trot c30_crawl c1; do
  timeout -k 10 180 python -u scripts/dropin_latency.py --shape $sh --mode fast >> gpurun_out/sd5/lat.jsonl 2> gpurun_out/sd5/lat.err || { echo "lat rc=$? $sh"; tail -5 gpurun_out/sd5/lat.err; exit 1; }
done
cut -c1-200 gpurun_out/sd5/lat.jsonl
