# Persistent solver diagnostics: one wave answering request after request
# (QPSWIFT_HIP_SERVE_LIFE_MS=10) with the default DPP wait states vs wait states inside
# every DPP asm (QPB_DPP_NOP=2), trot drop-in golden (scripts/serve_dbg.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export QPSWIFT_HIP_SERVE_LIFE_MS=10
for v in multi nop2 multi_b nop2_b; do
  ( case $v in nop2*) export QPB_WAVE_OPTS="QPB_DPP_NOP=2";; esac
    timeout -k 10 180 python -u scripts/serve_dbg.py > gpurun_out/sd2_$v.log 2>&1; echo "$v rc=$? bad=$(grep -c '"iters": [^5]' gpurun_out/sd2_$v.log)" )
done
