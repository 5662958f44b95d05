# Wave kernel MFMA G'WG check: controller-shape parity, timing, throughput.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py -m gpu -x -q -k "controller or c30 or C30 or wave" --timeout 120 --timeout-method thread > gpurun_out/mf_p.log 2>&1; rc=$?; tail -3 gpurun_out/mf_p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/wave_timing.py c30 > gpurun_out/wt.log 2>&1 || exit 1
grep "{" gpurun_out/wt.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); d=r['deltas']; print(r['iters'], r['total']); print({k:v for k,v in d.items() if k.startswith(('16','17','36','8->','9->'))})"
timeout -k 10 200 python -u scripts/tree_bench.py c30:wave:1 c30:wave:64 c30:wave:512 c30:wave:1024 c30:wave:8192 > gpurun_out/mf_b.log 2>&1; rc=$?; grep "{" gpurun_out/mf_b.log | cut -c1-170; exit $rc
