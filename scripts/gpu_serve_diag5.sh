# Persistent solver diagnostics: multi-request waves (QPSWIFT_HIP_SERVE_LIFE_MS=10), body
# inlined as shipped vs inlined with every kernel argument opaque per request
# (QPB_W_SERVE_OPQ=1), trot drop-in golden QP by QP (scripts/serve_dbg.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sd5; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
export QPSWIFT_HIP_SERVE_LIFE_MS=10
for v in inline opq1 opq2; do
  ( case $v in opq*) export QPB_WAVE_OPTS="QPB_W_SERVE_OPQ=1";; esac
    timeout -k 10 180 python -u scripts/serve_dbg.py > gpurun_out/sd5/$v.log 2> gpurun_out/sd5/$v.err; rc=$?
    fatal $rc $v; echo "$v rc=$rc bad=$(grep -c '"iters": [^5]' gpurun_out/sd5/$v.log) n=$(grep -c '"q"' gpurun_out/sd5/$v.log)"; exit $rc ) || exit 1
done
