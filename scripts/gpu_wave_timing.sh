# Phase stamps (QPB_W_TIMING=1) of the one-QP-per-wavefront kernel for the drop-in's
# AMD-ordered plans (C1, C30) and the leaves-first C30: where a Mehrotra iteration goes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/wave_timing.py c1:amd c30:amd c30 > gpurun_out/wave_timing.jsonl 2>gpurun_out/wave_timing.err; rc=$?
cut -c1-1500 gpurun_out/wave_timing.jsonl; tail -3 gpurun_out/wave_timing.err; exit $rc
