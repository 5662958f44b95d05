# Wave / row kernel knob A/B: a parity subset with the defaults, then for each variant
# (';'-separated QPB_WAVE_OPTS strings, "-" = defaults) the phase timing of the AMD-ordered
# and leaves-first C30 kernels, the drop-in C30 tick, the bench's headline (row kernel,
# 1 024 and 2^20 QPs) and shape legs, twice,
# interleaved.  Output: gpurun_out/wab/.
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/wab; mkdir -p $out; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_limits.py tests/test_serve.py -m gpu -q --timeout 120 --timeout-method thread -k "wave or dropin or serve or limits or row or kernel" > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $out/pytest.log)"; grep -E "^FAILED" $out/pytest.log | head -5; fatal $rc pytest; [ $rc = 0 ] || exit $rc
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for rep in 1 2; do for v in "${VS[@]}"; do
  o="$v"; [ "$o" = "-" ] && o=""; tag=$(echo "${v:-def}" | tr -c 'A-Za-z0-9=\n' '_')
  QPB_WAVE_OPTS="$o" timeout -k 10 300 python -u scripts/wave_timing.py c30:amd c30 > $out/t_${tag}_$rep.jsonl 2>> $out/err.log; rc=$?; fatal $rc timing; [ $rc = 0 ] || exit $rc
  QPB_WAVE_OPTS="$o" timeout -k 10 200 python -u scripts/dropin_latency.py --shape c30 --mode fast > $out/lat_${tag}_$rep.json 2>> $out/err.log; rc=$?; fatal $rc lat; [ $rc = 0 ] || exit $rc
  QPB_WAVE_OPTS="$o" timeout -k 10 400 python -u bench.py --no-cpu --no-mixed --steps 100 --warmup 10 > $out/b_${tag}_$rep.log 2>> $out/err.log; rc=$?; fatal $rc bench; [ $rc = 0 ] || exit $rc
  python3 - "$out" "$tag" "$rep" <<'PY'
import json, sys
out, tag, rep = sys.argv[1:]
t = [json.loads(l) for l in open(f"{out}/t_{tag}_{rep}.jsonl") if l.startswith("{")]
lat = [json.loads(l) for l in open(f"{out}/lat_{tag}_{rep}.json") if l.startswith("{")][-1]
b = [json.loads(l) for l in open(f"{out}/b_{tag}_{rep}.log") if l.startswith("{")][-1]
sh = {s["workload"][:18]: s.get("kernel_ms") or s.get("ms_per_step") for s in b["shapes"]}
print(json.dumps({"variant": tag, "rep": int(rep), "headline_us": round(b["roofline"]["kernel_ms"] * 1e3, 2),
                  "large_ms": round(b["large_batch"]["kernel_ms"], 3), "cycles": {x["shape"]: x["total"] for x in t},
                  "c30_tick_us": round(lat["gpu_us_median"], 1), "shapes_ms": sh}))
PY
done; done
