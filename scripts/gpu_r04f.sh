# Round 4: the cold (QP_SETUP init) resident wave is the one that goes wrong (r04e);
# bisect which kernel-argument group, hoisted out of its request loop, carries the fault:
# round 3's cold kernel (QPB_W_SIGOUT=0), multi-request waves for the cold server only,
# one argument group made opaque per request in each variant (QPB_W_SERVE_OPQ bit mask).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=
for k in 0 1 2 3 4 5 6 7 8; do V="$V g$k:QPB_WAVE_OPTS=QPB_W_SIGOUT=0+QPB_W_SERVE_OPQ=$((1 << (k + 1))),QPB_SERVE_DIAG_ONLY=cold"; done
bash scripts/gpu_serve_diag.sh $V all:QPB_WAVE_OPTS=QPB_W_SIGOUT=0+QPB_W_SERVE_OPQ=1,QPB_SERVE_DIAG_ONLY=cold \
  none:QPB_WAVE_OPTS=QPB_W_SIGOUT=0,QPB_SERVE_DIAG_ONLY=cold || exit 1
