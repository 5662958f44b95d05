# The 192-thread tree kernel (1 024 MPC QPs): 8 vs 4 prefetched descriptor rounds
# (QPB_T_PF; spilled registers 58 vs 14): time (interleaved) and FETCH / WRITE bytes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tpf; export TMPDIR=/tmp
: > gpurun_out/tpf/time.log
for rep in 1 2; do for v in "QPB_T_PF=8" "QPB_T_PF=4 QPB_T_XR=4" "QPB_T_PF=4 QPB_T_XR=8"; do
  QPB_TREE_OPTS="$v" timeout -k 10 300 python -u scripts/tree_bench.py mpc_h10:tree:1024 mpc_h10:tree:1 | sed "s/^/[$v] /" >> gpurun_out/tpf/time.log; rc=$?; [ $rc -eq 0 ] || exit $rc
done; done
for v in "QPB_T_PF=8" "QPB_T_PF=4 QPB_T_XR=4"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    tag=$(echo $v | tr ' =' '__')
    QPB_TREE_OPTS="$v" timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/tpf/${tag}_$c -o run -- python3 scripts/pmc_run.py --shape mpc_h10 --kernel tree --batch 1024 --reps 5 > gpurun_out/tpf/${tag}_$c.log 2>&1
    rc=$?; echo "$v $c rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
  done
done
cut -c1-220 gpurun_out/tpf/time.log
