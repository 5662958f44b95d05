# Persistent solver diagnostics: multi-request waves (QPSWIFT_HIP_SERVE_LIFE_MS=10) with
# the wave kernel as is, with every inline asm volatile (QPB_W_ASMV=1), and with the
# EXEC mask stored at the top of each request (QPB_W_EXECDBG=1; QPB_SERVE_DEBUG=1
# prints it), trot drop-in golden (scripts/serve_dbg.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export QPSWIFT_HIP_SERVE_LIFE_MS=10
for v in multi asmv execdbg; do
  ( case $v in asmv) export QPB_WAVE_OPTS="QPB_W_ASMV=1";; execdbg) export QPB_WAVE_OPTS="QPB_W_EXECDBG=1" QPB_SERVE_DEBUG=1;; esac
    timeout -k 10 180 python -u scripts/serve_dbg.py > gpurun_out/sd3_$v.log 2> gpurun_out/sd3_$v.err; echo "$v rc=$? bad=$(grep -c '"iters": [^5]' gpurun_out/sd3_$v.log)" )
done
