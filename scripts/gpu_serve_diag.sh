# Persistent solver, trot drop-in golden QP by QP (scripts/serve_dbg.py): one request
# per launch (default) vs one wave answering request after request (diagnostic mode).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in oneshot multi oneshot2 multi2; do
  ( case $v in multi*) export QPSWIFT_HIP_SERVE_LIFE_MS=10;; esac
    timeout -k 10 120 python -u scripts/serve_dbg.py > gpurun_out/sd_$v.log 2>&1; echo "$v rc=$? bad=$(grep -c '"iters": [^5]' gpurun_out/sd_$v.log)" )
done
