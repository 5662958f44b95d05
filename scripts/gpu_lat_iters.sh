# One-QP kernel latency against a fixed iteration count (tol 0, maxit K): the
# intercept is staging + kkt_initialize, the slope one Mehrotra iteration.
# Row form (default) vs one QP per wave (QPB_ROW=0) for C1; the AMD-ordered C30.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/lat_iters.jsonl
for r in "QPB_ROW=1" "QPB_ROW=0"; do
  env $r timeout -k 10 300 python -u scripts/lat_bench.py c1:amd:1:0::0 c1:amd:1:0::1 c1:amd:1:0::2 c1:amd:1:0::4 c1:amd:1:0::8 c1:amd:1024:0::8 \
    | sed "s/^/[$r] /" >> gpurun_out/lat_iters.jsonl || exit 1
done
timeout -k 10 300 python -u scripts/lat_bench.py c30:amd:1:0::0 c30:amd:1:0::2 c30:amd:1:0::4 c30:amd:1:0::8 >> gpurun_out/lat_iters.jsonl || exit 1
cut -c1-260 gpurun_out/lat_iters.jsonl
