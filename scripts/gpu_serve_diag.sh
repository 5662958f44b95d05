# Persistent-solver diagnostics in one driver (replaces round 3's gpu_serve_diag2-5 and
# gpu_serve_lat_opq): the trot drop-in golden QP by QP (scripts/serve_dbg.py) through
# multi-request resident waves (QPSWIFT_HIP_SERVE_LIFE_MS=10 + the QPB_SERVE_DIAG=1 guard),
# one process per variant.  Each argument is  name[:VAR=VAL[,VAR=VAL...]], e.g.
#   bash scripts/gpu_serve_diag.sh inline opq:QPB_WAVE_OPTS=QPB_W_SERVE_OPQ=1 prera:QPB_PRERA_OFF=1
# (QPB_WAVE_OPTS values with spaces: use '+' for the space).  oneshot:QPSWIFT_HIP_SERVE_LIFE_MS=0
# is the shipped mode.  LAT=1 also times the tick of every variant (scripts/dropin_latency.py).
# SEQ=1 runs QP_SETUP alone instead (scripts/serve_setup_seq.py: the cold wave's initial
# point per QP) and prints, per variant, '.' / 'X' against the variant named by SEQ_REF.
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/sd; mkdir -p $out; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
for spec in "$@"; do
  name=${spec%%:*}; vars=; [ "$spec" != "$name" ] && vars=${spec#*:}
  ( export QPSWIFT_HIP_SERVE_LIFE_MS=10 QPB_SERVE_DIAG=1
    IFS=,; for kv in $vars; do export "${kv%%=*}=$(echo "${kv#*=}" | tr + ' ')"; done; unset IFS
    if [ "${SEQ:-0}" = 1 ]; then
      timeout -k 10 120 python -u scripts/serve_setup_seq.py 2 > $out/$name.log 2> $out/$name.err; rc=$?
      fatal $rc $name; echo "$name [$vars] rc=$rc"; exit $rc
    fi
    timeout -k 10 180 python -u scripts/serve_dbg.py > $out/$name.log 2> $out/$name.err; rc=$?
    fatal $rc $name
    echo "$name [$vars] rc=$rc bad=$(grep -c '"ok": false' $out/$name.log) n=$(grep -c '"q"' $out/$name.log)"
    if [ "${LAT:-0}" = 1 ]; then
      for sh in c1 c30 c30_trot; do
        timeout -k 10 180 python -u scripts/dropin_latency.py --shape $sh --mode fast >> $out/$name.lat.jsonl 2>> $out/$name.err; rc=$?
        fatal $rc $name.lat; [ $rc = 0 ] || exit $rc
      done
    fi
    exit $rc ) || exit 1
done
if [ "${SEQ:-0}" = 1 ] && [ -n "$SEQ_REF" ]; then
  python3 - "$out" "$SEQ_REF" "$@" <<'PY'
import json, sys
out, ref = sys.argv[1], sys.argv[2]
names = [a.split(":")[0] for a in sys.argv[3:]]
L = {k: [json.loads(l)["init"] for l in open(f"{out}/{k}.log") if l.startswith("{")] for k in names}
for k, v in L.items():
    print(k, "".join("." if a == b else "X" for a, b in zip(v, L[ref])))
PY
fi
