# Round 4: row-kernel knobs A/B (headline + 2^20, interleaved; scripts/gpu_ab.sh), per-phase
# cycles per variant (scripts/row_timing.py), and the row-kernel parity tests per variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
export VARIANTS="${VARIANTS:--;QPB_R_EARLYGWG=1;QPB_R_RCP1=1;env:QPB_ROW_SPLIT=1}"
bash scripts/gpu_ab.sh || exit 1
IFS=';' read -ra VS <<< "$VARIANTS"
: > gpurun_out/row_timing.log
for v in "${VS[@]}"; do o="$v"; [ "$o" = "-" ] && o=""; ev=""
  case "$o" in env:*) ev="${o#env:}"; o="";; esac
  env $ev QPB_WAVE_OPTS="$o" timeout -k 10 200 python -u scripts/row_timing.py 1024 | sed "s/^/[$v] /" >> gpurun_out/row_timing.log; rc=$?; fatal $rc timing; [ $rc = 0 ] || exit 1
done
cut -c1-400 gpurun_out/row_timing.log
for v in "${VS[@]}"; do o="$v"; [ "$o" = "-" ] && continue; ev=""
  case "$o" in env:*) ev="${o#env:}"; o="";; esac
  env $ev QPB_WAVE_OPTS="$o" timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 120 --timeout-method thread \
     -k "wave_kernel_matches_oracle or ragged or large_batch or config1 or config2 or two_wave or fused_argmin" > gpurun_out/parity_knob.log 2>&1; rc=$?
  echo "parity [$v] rc=$rc $(tail -1 gpurun_out/parity_knob.log)"; fatal $rc parity
done
