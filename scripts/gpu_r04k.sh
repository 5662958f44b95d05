# Round 4: which new wave-kernel knob breaks the wave kernels (r04j): a short parity
# subset with each knob off in turn, and with all three off.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/k; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
for v in "none:" "noh0bf:QPB_W_H0BF=0" "nolskip:QPB_W_LSKIP=0" "notrunm:QPB_W_TRUNM=0" "alloff:QPB_W_H0BF=0 QPB_W_LSKIP=0 QPB_W_TRUNM=0"; do  # (QPB_W_TRUNM: an unmasked descending -L transpose, removed after this run: the compiler reorders per-lane stores)
  name=${v%%:*}; o=${v#*:}
  QPB_WAVE_OPTS="$o" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "wave_kernel_matches_oracle_in_its_order" > gpurun_out/k/$name.log 2>&1; rc=$?
  echo "$name [$o] rc=$rc $(tail -1 gpurun_out/k/$name.log)"; fatal $rc $name
done
exit 0
