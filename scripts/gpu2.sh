cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
timeout -k 10 600 python scripts/sweep.py --batch 1048576 --reps 5 --rounds 2 128:3 128:2 256:1 256:0 exact > gpurun_out/sweep.log 2> gpurun_out/sweep.err; rc=$?; echo "sweep rc=$rc"
