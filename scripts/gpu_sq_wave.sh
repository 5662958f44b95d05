# SQ / GRBM counter passes (kernel-trace only) of the wave and wide-row kernels the bench
# line names: the leaves-first controller shapes (1 024 QPs, wide row form), the controller
# call in AMD order (wave form) and leaves first (wide row form), 8 192 QPs
# -> scripts/sq_summary.py <dir> <out> wave | rowx.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sqw; export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MUL_F64"
G3="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
i=0
for grp in "$G1" "$G2" "$G3"; do i=$((i+1))
  timeout -k 10 -s KILL 400 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/sqw/p$i -o run -- python3 bench.py --no-cpu --no-mixed --steps 5 --warmup 2 --large-batch 4096 > gpurun_out/sqw/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; case $rc in 0) ;; *) tail -3 gpurun_out/sqw/p$i.log;; esac
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 scripts/sq_summary.py gpurun_out/sqw gpurun_out/sqw/sq_wave.json wave > gpurun_out/sqw/summary.log; echo "summary rc=$?"
python3 scripts/sq_summary.py gpurun_out/sqw gpurun_out/sqw/sq_rowx.json rowx > gpurun_out/sqw/summary_rowx.log; echo "rowx summary rc=$?"
