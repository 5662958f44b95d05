# Drop-in tick with Permut = NULL (AMD, the controller's call) against a caller-supplied
# leaves-first Permut (scripts/dropin_latency.py --permut): the drop-in GPU tests of both
# paths, then the four tick shapes per ordering, twice, interleaved; the CPU reference runs
# with the same Permut.  Output: gpurun_out/pm/lat.jsonl.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pm; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_dropin.py -m gpu -q --timeout 120 --timeout-method thread -k "leaves_first or fast_default" > gpurun_out/pm/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/pm/pytest.log)"; grep -E "^FAILED|Error" gpurun_out/pm/pytest.log | head -5; fatal $rc pytest; [ $rc = 0 ] || exit $rc
: > gpurun_out/pm/lat.jsonl
for rep in 1 2; do for pm in amd leaves; do for sh in c1 c30 c30_trot c30_crawl; do
  timeout -k 10 200 python -u scripts/dropin_latency.py --shape $sh --mode fast --permut $pm >> gpurun_out/pm/lat.jsonl 2>> gpurun_out/pm/lat.err; rc=$?
  fatal $rc lat; [ $rc = 0 ] || exit $rc
done; done; done
python3 - <<'PY'
import json
for l in open("gpurun_out/pm/lat.jsonl"):
    r = json.loads(l)
    print(r["shape"], r["permut"], "tick %.1f us" % r["gpu_us_median"], "device solve %.1f us" % r["serve_dev_solve_us"],
          "cpu ref %.1f us" % r.get("cpu_ref_us_median", 0), "x rel diff %.1e" % r.get("max_rel_x_diff", 0))
PY
