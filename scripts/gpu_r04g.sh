# Round 4: host-side probes on the failing configuration (round 3's cold kernel,
# multi-request waves for the cold server only) with the GPU code unchanged:
# QPB_SERVE_RECHECK=1 re-reads the results 0.5 ms after the answer (does any land
# late?), QPB_SERVE_PREDELAY_US holds each request back after its inputs were written.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=QPB_WAVE_OPTS=QPB_W_SIGOUT=0,QPB_SERVE_DIAG_ONLY=cold
bash scripts/gpu_serve_diag.sh rechk1:$B,QPB_SERVE_RECHECK=1 delay1:$B,QPB_SERVE_PREDELAY_US=300 \
  base1:$B rechk2:$B,QPB_SERVE_RECHECK=1 delay2:$B,QPB_SERVE_PREDELAY_US=300 base2:$B || exit 1
grep -h "recheck" gpurun_out/sd/rechk*.err | sort | uniq -c
exit 0
