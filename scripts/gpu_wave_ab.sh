# A/B of wave-kernel knobs on the controller QP (QPB_WAVE_OPTS variants from $VARIANTS, ';'-separated).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-;QPB_W_LDSB=0}"
for o in "${VS[@]}"; do
  echo "== $o"
  QPB_WAVE_OPTS="$o" timeout -k 10 200 python -u scripts/tree_bench.py ${CASES:-c30:wave:1 c30:wave:1024 c30:wave:8192} > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
  grep "{" gpurun_out/ab.log | cut -c1-125
done
