# MPC tree kernel (configs[3]): time at 1 024 and 1 QP, then HBM bytes per 1 024-QP
# launch (FETCH_SIZE / WRITE_SIZE passes, scripts/traffic.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tt; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/tree_bench.py mpc_h10:tree:1024 mpc_h10:tree:1 mpc_h10:tree:1024 mpc_h10:tree:8192 > gpurun_out/tt/time.log || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/tt/$c -o run -- python3 scripts/pmc_run.py --shape mpc_h10 --kernel tree --batch 1024 --reps 5 > gpurun_out/tt/$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cut -c1-220 gpurun_out/tt/time.log
