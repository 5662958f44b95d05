# band kernel (configs[3]) check: GPU parity file, cycles per phase / part, HIP-event
# timings at 1 / 1 024 / 8 192 MPC QPs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q --timeout 120 --timeout-method thread > gpurun_out/band_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/band_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
QPB_WAVE_OPTS="QPB_B_TIMING=1" timeout -k 10 120 python -u scripts/band_timing.py 1 1024 > gpurun_out/band_timing.jsonl 2>&1 || exit $?
QPB_WAVE_OPTS="QPB_B_TIMING=2" timeout -k 10 120 python -u scripts/band_timing.py 1 1024 >> gpurun_out/band_timing.jsonl 2>&1 || exit $?
timeout -k 10 200 python -u scripts/tree_bench.py mpc_h10:band:1 mpc_h10:band:1024 mpc_h10:band:8192 > gpurun_out/band_bench.jsonl 2>&1
echo "bench rc=$?"
