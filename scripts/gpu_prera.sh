# Round 3: (1) the full GPU suite with the pre-RA workaround OFF (QPB_PRERA_ON=1, every
# kernel recompiled with the default pipeline); (2) the round-2 source (worktree of
# 0a2aed1, its own library) with its default options, to confirm the old wrong iterate
# still reproduces on today's box.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
QPB_PRERA_ON=1 QPB_KCACHE=/tmp/kc_prera timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_prera_on.log 2>&1; rc=$?
echo "pytest (pre-RA on) rc=$rc"; tail -4 gpurun_out/pytest_prera_on.log
case $rc in 124|134|137|139) exit $rc;; esac
cd diag_r2wt && timeout -k 10 300 python -u scripts/diag_wave72.py base > ../gpurun_out/diag72_r2src.log 2>&1; rc2=$?; cd ..
echo "r2 source diag rc=$rc2"; cut -c1-300 gpurun_out/diag72_r2src.log
