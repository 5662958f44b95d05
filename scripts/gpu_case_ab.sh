# Kernel knob A/B on chosen plans, interleaved: CASES="c30:wave:1:amd c30:wave:8192:amd"
# (scripts/tree_bench.py case specs), VARIANTS="-;QPB_W_RCH=0" (QPB_WAVE_OPTS per variant,
# "-" = defaults), each variant in its own process, two repetitions.  DROPIN=c30 adds the
# drop-in tick (scripts/dropin_latency.py, Permut = NULL) per variant.
# Output: gpurun_out/case_ab.jsonl
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/case_ab.jsonl; : > $out
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for rep in 1 2; do for v in "${VS[@]}"; do
  o="$v"; [ "$o" = "-" ] && o=""
  QPB_WAVE_OPTS="$o" timeout -k 10 300 python -u scripts/tree_bench.py $CASES 2>/dev/null | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $out
  rc=${PIPESTATUS[0]}; echo "variant '$v' rep $rep rc=$rc"; [ $rc = 0 ] || exit $rc
  if [ -n "$DROPIN" ]; then
    QPB_WAVE_OPTS="$o" timeout -k 10 200 python -u scripts/dropin_latency.py --shape $DROPIN --mode fast 2>/dev/null | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $out
    rc=${PIPESTATUS[0]}; echo "dropin '$v' rep $rep rc=$rc"; [ $rc = 0 ] || exit $rc
  fi
done; done
