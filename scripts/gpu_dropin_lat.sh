# Drop-in per-tick latency (controller call pattern), default and with QPSWIFT_HIP_SETUP_INIT=0.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/dropin_latency.jsonl
for init in 1 0; do for sh in c1 c30 c30_trot c30_crawl; do
  QPSWIFT_HIP_SETUP_INIT=$init timeout -k 10 180 python -u scripts/dropin_latency.py --shape $sh --mode fast --setup-init $init >> gpurun_out/dropin_latency.jsonl 2>gpurun_out/dl.err || { echo "rc=$? $sh"; tail -5 gpurun_out/dl.err; exit 1; }
done; done
cut -c1-400 gpurun_out/dropin_latency.jsonl
