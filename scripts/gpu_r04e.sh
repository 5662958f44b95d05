# Round 4: which resident server carries the fault -- multi-request waves for the cold
# (QP_SETUP init) server only or the warm (QP_SOLVE) server only (QPB_SERVE_DIAG_ONLY),
# with round 3's cold kernel (QPB_W_SIGOUT=0); serve_dbg prints each QP's setup point.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=QPB_WAVE_OPTS=QPB_W_SIGOUT
bash scripts/gpu_serve_diag.sh coldonly_nosig:$O=0,QPB_SERVE_DIAG_ONLY=cold warmonly_nosig:$O=0,QPB_SERVE_DIAG_ONLY=warm \
  both_nosig:$O=0 both_sig oneshot_nosig:$O=0,QPSWIFT_HIP_SERVE_LIFE_MS=0 || exit 1
