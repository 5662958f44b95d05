# Attribution of the tree kernel's step chain on MPC (fixed 6 iterations, tol 0):
# each QPB_T_EXP variant removes one part of every step (timing only: wrong results).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/texp.jsonl
for v in "" "QPB_T_EXP=2" "QPB_T_EXP=3" "QPB_T_EXP=4" "QPB_T_EXP=5" "QPB_T_DEPTH=4" ""; do
  QPB_TREE_OPTS="$v" timeout -k 10 300 python -u scripts/lat_bench.py mpc_h10:own:1:0:tree:6 mpc_h10:own:1024:0:tree:6 2>gpurun_out/texp.err | sed "s/^/{\"opts\": \"$v\", \"r\": /; s/$/}/" >> gpurun_out/texp.jsonl
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "variant '$v' rc=$rc"; tail -5 gpurun_out/texp.err; exit $rc; }
done
cat gpurun_out/texp.jsonl | cut -c1-230
