# The 192-thread tree kernel (1 024 MPC QPs) with and without QPB_T_PDUP: time and
# FETCH_SIZE / WRITE_SIZE (its spilled registers live in scratch memory).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tta; export TMPDIR=/tmp
for v in "QPB_T_PDUP=1" "QPB_T_PDUP=0"; do
  QPB_TREE_OPTS="$v" timeout -k 10 300 python -u scripts/tree_bench.py mpc_h10:tree:1024 mpc_h10:tree:1024 | sed "s/^/[$v] /" >> gpurun_out/tta/time.log; rc=$?; [ $rc -eq 0 ] || exit $rc
  for c in FETCH_SIZE WRITE_SIZE; do
    QPB_TREE_OPTS="$v" timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/tta/${v#QPB_T_}_$c -o run -- python3 scripts/pmc_run.py --shape mpc_h10 --kernel tree --batch 1024 --reps 5 > gpurun_out/tta/${v#QPB_T_}_$c.log 2>&1
    rc=$?; echo "$v $c rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
  done
done
cat gpurun_out/tta/time.log | cut -c1-200
