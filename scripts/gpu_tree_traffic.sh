# FETCH_SIZE / WRITE_SIZE of the tree kernel on MPC QPs: the 256-thread form
# (no spilled registers) at 512 QPs vs the 192-thread form (spills) at 1 024.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tt; export TMPDIR=/tmp
for b in 512 1024; do for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/tt/b${b}_$c -o run -- python3 scripts/pmc_run.py --shape mpc_h10 --kernel tree --batch $b --reps 5 > gpurun_out/tt/b${b}_$c.log 2>&1
  rc=$?; echo "tree traffic $b $c rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
done; done
