# A/B: DPP asm padded by qpb_hazard's asm_fixup (default) vs unpadded (QPB_NO_ASM_FIXUP=1).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/ab_fixup.jsonl
for r in 1 2; do for v in "" "QPB_NO_ASM_FIXUP=1"; do
  env $v timeout -k 10 300 python bench.py --no-shapes --no-cpu --no-mixed --steps 300 > gpurun_out/ab1.log 2>&1 || { echo "bench rc=$? ($v)"; tail -5 gpurun_out/ab1.log; exit 1; }
  python -c "import json,sys; r=json.loads([l for l in open('gpurun_out/ab1.log') if l.startswith('{')][-1]); print(json.dumps({'variant': '$v' or 'padded', 'value': r['value'], 'kernel_ms': r['roofline']['kernel_ms'], 'large_value': r['large_batch']['value'], 'large_kernel_ms': r['large_batch']['kernel_ms']}))" >> gpurun_out/ab_fixup.jsonl
done; done
cat gpurun_out/ab_fixup.jsonl
