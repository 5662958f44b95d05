# SQ / GRBM counter passes (kernel-trace only) of the row kernel at the headline
# batch (1 024 C1 QPs) and at 2^20 QPs: the evidence for roofline.bound.
cd "$GRAFT_REPO_ROOT"; D=${SQDIR:-gpurun_out/sq}; mkdir -p $D; export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MUL_F64"
G3="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
for b in "1024 50" "1048576 2"; do set -- $b
  i=0
  for grp in "$G1" "$G2" "$G3"; do i=$((i+1))
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $D/b$1_p$i -o run -- python3 scripts/pmc_run.py --batch $1 --reps $2 > $D/b$1_p$i.log 2>&1
    rc=$?; echo "batch $1 pass $i rc=$rc"; case $rc in 0) ;; *) tail -3 $D/b$1_p$i.log;; esac
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
