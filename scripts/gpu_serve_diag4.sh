# Persistent solver diagnostics: multi-request waves (QPSWIFT_HIP_SERVE_LIFE_MS=10) with
# the request body inlined into the loop (as shipped) vs the body as a noinline call
# (QPB_W_SERVE_CALL=1: no register allocation spans the request loop), trot drop-in
# golden QP by QP (scripts/serve_dbg.py), then the tick latency of the call form.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sd4; export TMPDIR=/tmp
# a fault, abort or time limit ends this call: gpu_round3.sh does not start after it
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; touch gpurun_out/FATAL; exit $1;; esac; }
export QPSWIFT_HIP_SERVE_LIFE_MS=10
for v in inline call1 call2 call3; do
  ( case $v in call*) export QPB_WAVE_OPTS="QPB_W_SERVE_CALL=1";; esac
    timeout -k 10 180 python -u scripts/serve_dbg.py > gpurun_out/sd4/$v.log 2> gpurun_out/sd4/$v.err; rc=$?
    fatal $rc $v; echo "$v rc=$rc bad=$(grep -c '"iters": [^5]' gpurun_out/sd4/$v.log) n=$(grep -c '"q"' gpurun_out/sd4/$v.log)"; exit $rc ) || exit 1
done
: > gpurun_out/sd4/lat.jsonl
for sh in c30 c30_trot c30_crawl c1; do
  QPB_WAVE_OPTS="QPB_W_SERVE_CALL=1" timeout -k 10 180 python -u scripts/dropin_latency.py --shape $sh --mode fast >> gpurun_out/sd4/lat.jsonl 2> gpurun_out/sd4/lat.err || { rc=$?; fatal $rc lat_$sh; echo "lat rc=$rc $sh"; tail -5 gpurun_out/sd4/lat.err; exit 1; }
done
cut -c1-300 gpurun_out/sd4/lat.jsonl
