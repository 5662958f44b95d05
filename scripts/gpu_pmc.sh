# PMC passes (kernel-trace only, no sys/runtime traces) for one kernel variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
V="${VARIANT:-128:3}"; if [ "$V" != "wave" ]; then export QPB_WG="${V%%:*}" QPB_LDS="${V##*:}"; fi
GROUPS_MAX="${GROUPS_MAX:-6}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1)); [ $i -gt $GROUPS_MAX ] && break
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/pmc_run.py ${PMC_ARGS} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
