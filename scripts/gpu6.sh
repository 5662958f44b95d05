cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python scripts/sweep.py --batch 1048576 --reps 5 --rounds 2 64:4 128:2 > gpurun_out/sweep.log 2> gpurun_out/sweep.err; echo "sweep rc=$?"
rm -rf gpurun_out/pmc; VARIANT=64:4 bash scripts/gpu_pmc.sh
