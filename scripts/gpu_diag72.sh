# Round 3: does the 7.2 wrong-iterate reproduce with the current source, padded or not?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/diag_wave72.py padded unpadded prera_on prera_on_unpadded row_knobs > gpurun_out/diag72.log 2>&1; rc=$?
cut -c1-400 gpurun_out/diag72.log; exit $rc
