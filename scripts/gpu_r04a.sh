# Round 4, first GPU call: parity suite (configs first), smoke, the multi-request
# persistent-wave bisection (scripts/gpu_serve_diag.sh), then the bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -3 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; fatal $rc smoke
O=QPB_WAVE_OPTS=QPB_W_SERVE_OPQ
bash scripts/gpu_serve_diag.sh oneshot:QPSWIFT_HIP_SERVE_LIFE_MS=0 inline prera:QPB_PRERA_OFF=1 opq:$O=1 \
  g0:$O=2 g1:$O=4 g2:$O=8 g3:$O=16 g4:$O=32 g5:$O=64 g6:$O=128 g7:$O=256 g8:$O=512 inline2 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.log; fatal $rc bench
