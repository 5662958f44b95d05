# SQ counter passes (kernel-trace only) of the band kernel on configs[3] (1 024 MPC-horizon
# QPs and one QP), then FETCH_SIZE / WRITE_SIZE passes at 1 024 and 8 192 QPs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sqb gpurun_out/trb; export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MUL_F64"
G3="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
for b in "1024 5" "1 5"; do set -- $b
  i=0
  for grp in "$G1" "$G2" "$G3"; do i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/sqb/b$1_p$i -o run -- python3 scripts/pmc_run.py --shape mpc_h10 --kernel band --batch $1 --reps $2 > gpurun_out/sqb/b$1_p$i.log 2>&1
    rc=$?; echo "band batch $1 pass $i rc=$rc"; case $rc in 0) ;; *) tail -3 gpurun_out/sqb/b$1_p$i.log;; esac
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
for b in 1024 8192; do
  for cn in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $cn --kernel-trace --output-format csv -d gpurun_out/trb/b${b}_$cn -o run -- python3 scripts/pmc_run.py --shape mpc_h10 --kernel band --batch $b --reps 3 > gpurun_out/trb/b${b}_$cn.log 2>&1
    rc=$?; echo "band batch $b $cn rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
