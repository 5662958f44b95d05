cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/wave_timing.py c30 c30:amd > gpurun_out/wt.jsonl 2>&1 && QPB_WAVE_OPTS="QPB_W_BLK=0" timeout -k 10 200 python -u scripts/wave_timing.py c30:amd >> gpurun_out/wt.jsonl 2>&1; cat gpurun_out/wt.jsonl | tail -5
