# Kernel-only latency of single-QP launches, a few knob variants (VARIANTS, ';'-separated).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:--}"
: > gpurun_out/lat.jsonl
for v in "${VS[@]}"; do o="$v"; [ "$o" = "-" ] && o=""
  QPB_WAVE_OPTS="$o" timeout -k 10 300 python -u scripts/lat_bench.py ${CASES:-c30:amd:1 c30:own:1 c30_trot:amd:1 c1:own:1 c1:own:1024} >> gpurun_out/lat.jsonl 2>gpurun_out/lat.err || { tail -5 gpurun_out/lat.err; exit 1; }
done
cat gpurun_out/lat.jsonl
