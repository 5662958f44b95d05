cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/sweep.py --batch 1024 --reps 20 --rounds 2 wave wave:RDLDS=1 wave:GATHER=15 > gpurun_out/sweep5.log 2>&1 || { tail -20 gpurun_out/sweep5.log; exit 1; }
cat gpurun_out/sweep5.log | grep variant
VARIANTS="-;QPB_R_RDLDS=1" bash scripts/gpu_ab.sh || exit 1
SQDIR=gpurun_out/sq_def bash scripts/gpu_sq.sh
QPB_WAVE_OPTS="QPB_R_GATHER=15 QPB_R_PIVLDS=1" SQDIR=gpurun_out/sq_gather bash scripts/gpu_sq.sh
