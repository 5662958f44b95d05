# Drop-in A/B: the drop-in / persistent-solver GPU tests with the defaults, then the
# per-tick latency (scripts/dropin_latency.py, fast mode) of C1 and the three C30 shapes
# for each variant (';'-separated env assignments, "-" = defaults), twice, interleaved.
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/dab; mkdir -p $out; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_dropin.py tests/test_serve.py tests/test_c_caller.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $out/pytest.log)"; grep -E "^FAILED" $out/pytest.log | head -5; fatal $rc pytest; [ $rc = 0 ] || exit $rc
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for rep in 1 2; do for v in "${VS[@]}"; do
  ev=""; [ "$v" != "-" ] && ev="$v"; tag=$(echo "${v}" | tr -c 'A-Za-z0-9=\n' '_')
  for sh in c1 c30 c30_trot c30_crawl; do
    env $ev timeout -k 10 200 python -u scripts/dropin_latency.py --shape $sh --mode fast > $out/lat_${tag}_${rep}_$sh.json 2>> $out/err.log; rc=$?; fatal $rc lat; [ $rc = 0 ] || exit $rc
    python3 -c "
import json
r=[json.loads(l) for l in open('$out/lat_${tag}_${rep}_$sh.json') if l.startswith('{')][-1]
print(json.dumps({'variant': '$tag', 'rep': $rep, 'shape': '$sh', 'tick_us': round(r['gpu_us_median'],1), 'setup_us': round(r['gpu_setup_us'],1), 'solve_us': round(r['gpu_solve_us'],1), 'dev_setup_us': r.get('serve_dev_setup_us'), 'dev_solve_us': r.get('serve_dev_solve_us'), 'rel_x': r.get('max_rel_x_diff')}))"
  done
done; done
