# Cost attribution of the wave kernel (timing-only builds, wrong results): each phase
# skipped in turn (QPB_W_ABL: 1 LDL' 2 G'WG 4 solve chains 8 residual products
# 16 transpose), fixed 8 iterations (tol 0), one QP (latency) and 1 024 QPs (throughput),
# AMD-ordered and leaves-first 30/68/18 (scripts/lat_bench.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/wave_abl.jsonl
for a in 0 1 2 4 8 16; do
  QPB_WAVE_OPTS="QPB_W_ABL=$a" timeout -k 10 300 python -u scripts/lat_bench.py c30:amd:1:0:wave1:8 c30:amd:1024:0:wave:8 c30:own:1:0:wave1:8 c30:own:1024:0:wave:8 >> gpurun_out/wave_abl.jsonl 2>> gpurun_out/wave_abl.err; rc=$?
  echo "abl=$a rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
python3 -c "
import json
for l in open('gpurun_out/wave_abl.jsonl'):
    r=json.loads(l); print(r['opts'], r['case'], round(r['us_per_launch'],1))"
