# lat_bench.py CASES under several environment settings (ENVS: ';'-separated, "-" = none).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra ES <<< "${ENVS:--}"
: > gpurun_out/el.jsonl
for e in "${ES[@]}"; do ee="$e"; [ "$ee" = "-" ] && ee=""
  env $ee timeout -k 10 300 python -u scripts/lat_bench.py $CASES > gpurun_out/el_one.jsonl 2>gpurun_out/el.err || { tail -5 gpurun_out/el.err; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/el_one.jsonl'):
    r=json.loads(l); r['env']=sys.argv[1]; print(json.dumps(r))" "$e" >> gpurun_out/el.jsonl
done
python3 -c "
import json
for l in open('gpurun_out/el.jsonl'):
    r=json.loads(l); print(r['env'], r['case'], round(r['us_per_launch'],1), r['mean_iters'])"
