# Round 4: QP_SETUP alone through the cold persistent wave (scripts/serve_setup_seq.py):
# round 3's cold kernel (QPB_W_SIGOUT=0) multi-request vs one request per wave, and
# today's cold kernel multi-request.
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/ss; mkdir -p $out; export TMPDIR=/tmp
run() { name=$1; shift
  ( export QPB_SERVE_DIAG=1 "$@"; timeout -k 10 120 python -u scripts/serve_setup_seq.py 2 > $out/$name.log 2> $out/$name.err ); rc=$?
  echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
run multi_nosig QPSWIFT_HIP_SERVE_LIFE_MS=10 QPB_WAVE_OPTS=QPB_W_SIGOUT=0 || exit 1
run oneshot_nosig QPSWIFT_HIP_SERVE_LIFE_MS=0 QPB_WAVE_OPTS=QPB_W_SIGOUT=0 || exit 1
run multi_sig QPSWIFT_HIP_SERVE_LIFE_MS=10 || exit 1
python3 - <<'PY'
import json
L = {k: [json.loads(l)["init"] for l in open(f"gpurun_out/ss/{k}.log") if l.startswith("{")] for k in ("multi_nosig", "oneshot_nosig", "multi_sig")}
ref = L["oneshot_nosig"]
for k, v in L.items():
    print(k, "".join("." if a == b else "X" for a, b in zip(v, ref)))
PY
