# Round 4: the advisor's pre-RA check on the failing resident setup kernel (round 3's
# cold kernel, multi-request waves for the cold server only) with
# -amdgpu-enable-pre-ra-optimizations=0 (QPB_PRERA_OFF=1), then the closing run.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=QPB_WAVE_OPTS=QPB_W_SIGOUT=0,QPB_SERVE_DIAG_ONLY=cold
bash scripts/gpu_serve_diag.sh preraoff1:$B,QPB_PRERA_OFF=1 preraoff2:$B,QPB_PRERA_OFF=1 base:$B || exit 1
bash scripts/gpu_r04_final.sh
