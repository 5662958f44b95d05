# Round 3: the 7.2 wrong iterate with today's source: which source change removed the trigger?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/diag_wave72.py ${DIAG_VARIANTS} > gpurun_out/diag72b.log 2>&1; rc=$?
cut -c1-600 gpurun_out/diag72b.log; exit $rc
