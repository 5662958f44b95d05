# Round-3 final counters: HBM bytes (FETCH_SIZE / WRITE_SIZE passes) of the row kernel
# at 1 024 and 2^20 C1 QPs and of the MPC tree kernel at 1 024, then the row kernel's
# SQ / GRBM passes (scripts/gpu_sq.sh).  Kernel-trace only, one counter group per pass.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fp; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  for b in "1024 50" "1048576 2"; do set -- $b
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/fp/row_${c}_$1 -o run -- python3 scripts/pmc_run.py --batch $1 --reps $2 > gpurun_out/fp/row_${c}_$1.log 2>&1
    rc=$?; echo "row $c $1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/fp/tree_$c -o run -- python3 scripts/pmc_run.py --shape mpc_h10 --kernel tree --batch 1024 --reps 5 > gpurun_out/fp/tree_$c.log 2>&1
  rc=$?; echo "tree $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_sq.sh
