# wide row kernel knob A/B, interleaved: VARIANTS="-;QPB_X_WLDS=1;..." (QPB_WAVE_OPTS per
# variant), HIP-event timings of the stance shape at 1, 1 024 and 8 192 QPs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; out=gpurun_out/rowx_ab.jsonl; : > $out
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for rep in 1 2; do
  for v in "${VS[@]}"; do
    opts=""; [ "$v" != "-" ] && opts="$v"
    QPB_WAVE_OPTS="$opts" timeout -k 10 120 python -u scripts/tree_bench.py c30:wave:1 c30:wave:1024 c30:wave:8192 2>/dev/null | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $out
    rc=${PIPESTATUS[0]}; echo "variant $v rep $rep rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
