# Wave-kernel parity (controller shapes, drop-in) + phase timing + drop-in C30 latency.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_assemble.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "wave or dropin or controller or assemble" > gpurun_out/wc_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/wc_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/wave_timing.py c30 c30:amd > gpurun_out/wt.jsonl 2>&1 || exit 1
: > gpurun_out/wc_dropin.jsonl
for sh in c30 c30_trot; do timeout -k 10 200 python -u scripts/dropin_latency.py --shape $sh --mode fast >> gpurun_out/wc_dropin.jsonl 2>gpurun_out/wc_dl.err || exit 1; done
cat gpurun_out/wc_dropin.jsonl
