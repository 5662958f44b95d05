# Round 4: (1) the multi-request wave with round 3's cold kernel restored (QPB_W_SIGOUT=0,
# code-identical to round 3's) vs today's, three processes each, serve counters printed;
# tick latency of both modes (LAT=1); (2) the row-kernel knob A/B (scripts/gpu_r04b.sh).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=QPB_WAVE_OPTS=QPB_W_SIGOUT
bash scripts/gpu_serve_diag.sh inline nosig1:$O=0 nosig2:$O=0 inline2 || exit 1
for f in inline nosig1 nosig2 inline2; do echo "$f $(tail -1 gpurun_out/sd/$f.log)"; done
LAT=1 bash scripts/gpu_serve_diag.sh multi || exit 1
for f in multi; do python3 -c "
import json,sys
for l in open('gpurun_out/sd/$f.lat.jsonl'):
    r=json.loads(l); print('$f', {k: r[k] for k in r if k in ('shape','gpu_us_median','gpu_us_p99','serve_requests','serve_launches','serve_dev_solve_us','cpu_ref_us_median','max_rel_x_diff')})"; done
bash scripts/gpu_r04b.sh
