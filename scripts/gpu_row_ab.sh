# Row-kernel A/B (headline + 2^20, interleaved) and per-phase cycles for a knob set
# VARIANTS (';'-separated QPB_WAVE_OPTS, "-" = defaults); then the GPU test suite.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh || exit $?
IFS=';' read -ra VS <<< "${VARIANTS:--}"
: > gpurun_out/row_timing.log
for v in "${VS[@]}"; do o="$v"; [ "$o" = "-" ] && o=""
  QPB_WAVE_OPTS="$o" timeout -k 10 200 python -u scripts/row_timing.py 1024 | sed "s/^/[$v] /" >> gpurun_out/row_timing.log || exit 1
done
[ -n "$NO_TESTS" ] || bash scripts/gpu_pytest.sh
