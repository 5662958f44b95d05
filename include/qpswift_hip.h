/*
 * qpswift_hip.h -- batched qpSWIFT interior-point solver for AMD MI355X (gfx950).
 *
 * C ABI only: plain pointers and sizes, no C++ or torch types.  This header is
 * the NEW batched entry point behind the reference's per-tick solve; the
 * source/ABI-compatible single-QP drop-in (QP_SETUP / QP_SETUP_dense / QP_SOLVE /
 * QP_CLEANUP / QP_CLEANUP_dense) is declared in qpSWIFT.h next to this file.
 *
 * Reference interface each entry point replaces (paths under
 * /root/reference/dogbot_controller/):
 *   qpb_plan_create   pattern half of QP_SETUP (src/qpSWIFT/qpSWIFT.c:60-234):
 *                     transposes, KKT assembly (Auxilary.c:71-181), AMD ordering
 *                     (qpSWIFT.c:416-440) and LDL_symbolic (ldl.c:187-240), done
 *                     once per sparsity pattern instead of once per tick.
 *   qpb_solve         value half of QP_SETUP (kkt_initialize, Auxilary.c:992-1089)
 *                     + QP_SOLVE (qpSWIFT.c:473-644) for B independent QPs that
 *                     share the plan's pattern, in one HIP launch.
 *   qpb_plan_destroy  QP_CLEANUP (qpSWIFT.c:661-737) for the pattern state.
 *
 * Data layout (device memory, "tiled SoA", tile = 64 QPs = one wavefront): an
 * array holding nv values per QP stores value j of QP q at
 *       X[(q / 64) * nv * 64 + j * 64 + q % 64]
 * i.e. the batch is cut into tiles of 64 QPs and each tile is an [nv][64] block;
 * buffers hold ceil(B/64) tiles.  (For nv = 1 this is a plain [B] array.)
 *   P  nv = nnz(P): values of the P pattern given at plan creation (full, or
 *      upper triangle with QPB_P_UPPER), in CSC order
 *   A  nv = nnz(A) (may be NULL when p == 0),   G  nv = nnz(G)
 *   c nv = n, h nv = m, b nv = p
 *   x nv = n, y nv = p, z nv = m, s nv = m           (outputs)
 *   flag [B] (QP_OPTIMAL 0 / QP_MAXIT 2), iters [B], fval [B]
 *   stats  optional, nv = 6: n_rx, n_ry, n_rz, n_mu, alpha_p, alpha_d
 * All pointers passed to qpb_solve are DEVICE pointers.  The call is asynchronous
 * on `stream` (a hipStream_t, NULL = default stream) and graph-capturable.
 *
 * Errors: every function returns 0 on success or a negative QPB_E* code and
 * records a message readable with qpb_last_error(); nothing is printed.
 */
#ifndef QPSWIFT_HIP_H
#define QPSWIFT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qpb_plan qpb_plan;

/* qpb_plan_create flags */
#define QPB_P_FULL   0x0   /* P pattern holds both triangles (QP_SETUP semantics) */
#define QPB_P_UPPER  0x1   /* P pattern is the upper triangle (symmetric P)        */
#define QPB_EXACT    0x10  /* bit-faithful arithmetic: IEEE division, no FMA       */
/* Ordering when perm == NULL.  Default (none of these): ours -- leaves first
 * (z rows, y rows, then x in natural order) for n, p <= 64, m <= 256 (the row
 * kernel's elimination for the contact-force shapes; a dense block of n rows for
 * the wave kernel), else exact minimum degree.  Either agrees with qpSWIFT to
 * 1e-6 at its default tolerance; loosely converged iterates (the controller's
 * tol 1e-2) depend on which pivots get regularised, i.e. on the ordering --
 * QPB_ORDER_AMD reproduces qpSWIFT's. */
#define QPB_ORDER_AMD    0x20  /* the reference's AMD (qpSWIFT.c:424-440, amd_l_defaults):
                                  QP_SETUP's Permut = NULL -- the same pivots, hence the
                                  same regularised pivots, as qpSWIFT                 */
#define QPB_ORDER_MINDEG 0x40  /* exact minimum degree, lowest-index ties             */
#define QPB_ORDER_LEAVES 0x80  /* z rows, y rows, then x rows in natural order        */
#define QPB_KERNEL_LANE 0x100  /* always the lane kernel (one QP per lane)         */
#define QPB_KERNEL_WAVE 0x200  /* always the wave kernel (wave or row form)         */
#define QPB_KERNEL_NOROW 0x400 /* wave kernel in its one-QP-per-wavefront form even
                                  where the row form (four QPs per wavefront) fits */
#define QPB_KERNEL_TREE 0x800  /* always the tree kernel (one QP per workgroup,
                                  level-scheduled sparse LDL'; any pattern)        */
#define QPB_KERNEL_BAND 0x1000 /* the band kernel for cold and warm solves (one QP per
                                  wavefront, block-tridiagonal LDL' over the stages of a
                                  multi-stage pattern, e.g. an MPC horizon; a plan without
                                  that structure: tree) */

/* error codes */
#define QPB_OK        0
#define QPB_EINVAL   -1
#define QPB_ENOMEM   -2
#define QPB_EHIP     -3
#define QPB_ECOMPILE -4
#define QPB_ESHAPE   -5

typedef struct qpb_settings {
    long   maxit;     /* default 100  (GlobalOptions.h:46) */
    double reltol;    /* default 1e-6 (GlobalOptions.h:47); controller uses 1e-2 */
    double abstol;    /* default 1e-6 (GlobalOptions.h:48) */
    double sigma_d;   /* 0 for QP_SETUP_dense (qpSWIFT.c:334) */
} qpb_settings;

typedef struct qpb_plan_info {
    long n, m, p, N;             /* N = n + m + p (KKT order) */
    long nnzP, nnzA, nnzG;       /* value counts per QP */
    long nnzK, lnz;              /* nnz of the KKT and of its L factor */
    long fac_updates, fac_divs;  /* LDL numeric op counts per factorisation */
    int  ordering;               /* 0 caller permutation, 1 own minimum degree, 2 the reference's AMD,
                                    3 own leaves-first (z rows, y rows, x rows) */
    int  exact;
    uint64_t hash;               /* pattern + permutation hash */
    int  wave_ok;                /* plan can use the wave-cooperative kernel */
    long wave_max_batch;         /* qpb_solve uses it for B <= this (-1: always) */
    int  wave_qpw;               /* QPs per wavefront of that kernel: 1 wave form, 4 row form */
    int  tree_ok;                /* plan can use the tree kernel (one QP per workgroup) */
    int  large_kernel;           /* kernel used beyond the wave kernel's range: 1 lane, 2 wave, 3 tree,
                                    4 band (cold solves; warm solves of such plans: tree) */
} qpb_plan_info;

void qpb_default_settings(qpb_settings *st);

int  qpb_plan_create(qpb_plan **plan, long n, long m, long p, int flags,
                     const long *Pjc, const long *Pir,
                     const long *Ajc, const long *Air,
                     const long *Gjc, const long *Gir,
                     const long *perm /* length n+m+p, or NULL: own / QPB_ORDER_* */);
void qpb_plan_destroy(qpb_plan *plan);
int  qpb_plan_get_info(const qpb_plan *plan, qpb_plan_info *info);
int  qpb_plan_get_perm(const qpb_plan *plan, long *perm /* [N] */);
/* Host-side AMD ordering of an n x n CSC pattern (A + A' ordered, diagonal
 * ignored; unsorted columns / duplicates allowed): replaces amd_l_order with
 * amd_l_defaults (src/qpSWIFT/amd_order.c:21-199, include/qpSWIFT/amd.h:339-348)
 * and writes the same permutation.  Returns 0 (OK), 1 (OK, input was unsorted or
 * had duplicates) or QPB_EINVAL.  Needs no GPU. */
int  qpb_amd_order(long n, const long *Ap, const long *Ai, long *perm);
/* Generated HIP source of the plan's kernel; returns its length (copies at most
 * cap-1 bytes plus a NUL when buf is non-NULL). */
long qpb_plan_source(const qpb_plan *plan, char *buf, long cap);
long qpb_plan_wave_source(const qpb_plan *plan, char *buf, long cap);
long qpb_plan_tree_source(const qpb_plan *plan, char *buf, long cap);
/* Name of the kernel qpb_solve launches for a batch of B (as the profilers list
 * it); returns its length, copies at most cap-1 bytes plus a NUL. */
long qpb_plan_kernel_name(const qpb_plan *plan, long B, char *buf, long cap);
/* The tree kernel's plan tables (uploaded once per device; exposed for tests):
 * returns their size in bytes, copies at most cap bytes when buf is non-NULL. */
long qpb_plan_tree_tables(const qpb_plan *plan, void *buf, long cap);
/* Compile the plan's kernels for gfx950 (hiprtc) or fetch them from the
 * code-object cache; needs no GPU.  qpb_solve calls this implicitly. */
int  qpb_plan_compile(qpb_plan *plan);
/* The same for the warm-solve variant qpb_solve_warm launches for a batch of B
 * (compiled on first use otherwise). */
int  qpb_plan_compile_warm(qpb_plan *plan, long B);
/* Compile (or fetch from the code-object cache) the persistent forms of the plan's
 * one-QP kernel that the drop-in's device solves use (include/qpSWIFT.h): 0, or 1
 * when that kernel (tree or lane) has none. */
int  qpb_plan_compile_serve(qpb_plan *plan);

int  qpb_solve(qpb_plan *plan, long B,
               const double *P, const double *A, const double *G,
               const double *c, const double *h, const double *b,
               const qpb_settings *st,
               double *x, double *y, double *z, double *s,
               int *flag, int *iters, double *fval, double *stats,
               void *stream);

/* qpb_solve followed by qpb_argmin into best (DEVICE, >= 2 doubles; receives
 * {fval, index}): one call per control step. */
int  qpb_solve_best(qpb_plan *plan, long B,
                    const double *P, const double *A, const double *G,
                    const double *c, const double *h, const double *b,
                    const qpb_settings *st,
                    double *x, double *y, double *z, double *s,
                    int *flag, int *iters, double *fval, double *stats,
                    double *best, void *stream);

/* Warm solve: QP_SOLVE called again on the same QP objects.  The reference's
 * QP_SOLVE (qpSWIFT.c:473-644) never re-initialises: it continues from the
 * object's x, y, z, s, stats->IterationCount and options->sigma, runs at most
 * maxit further iterations, and sets QP_MAXIT only when IterationCount reaches
 * exactly maxit (:598-601), otherwise leaving stats->Flag as it was.  Here every
 * QP q continues from x, y, z, s, iters[q] and flag[q] as they are in the (in/out)
 * arrays and from sigma[q] (DEVICE, [B]; in/out: receives the last sigma).  A cold
 * qpb_solve with maxit = 0 leaves kkt_initialize's point in x, y, z, s (what
 * QP_SETUP leaves in the QP, qpSWIFT.c:447); warm solves from there with
 * iters = 0, flag = QP_FATAL and sigma = 100 reproduce a cold solve. */
int  qpb_solve_warm(qpb_plan *plan, long B,
                    const double *P, const double *A, const double *G,
                    const double *c, const double *h, const double *b,
                    const qpb_settings *st,
                    double *x, double *y, double *z, double *s,
                    int *flag, int *iters, double *fval, double *stats,
                    double *sigma, void *stream);

/* Lowest-fval optimal QP of a batch (device-side reduction): writes
 * {fval, index} of the minimum over q with flag[q] == 0 (ties -> lowest index;
 * none -> {+inf, -1}) to out2 (device, 2 doubles; the index as a double). */
int  qpb_argmin(long B, const double *fval, const int *flag, double *out2, void *stream);

/* The multi-GPU gather's payload: out[0..1] = best {fval, index}
 * (from qpb_solve_best / qpb_argmin), out[2..2+n) = x of that QP read from the
 * tiled outputs x (nv = n, B QPs), NaN when index is -1.  One small launch on
 * `stream`; all_gather the 2 + n doubles of every rank (RCCL) and every rank
 * holds the global winner's solution.  DEVICE pointers. */
int  qpb_winner(const double *best, const double *x, long n, long B, double *out, void *stream);

/* On-device assembly of contact-force QPs (the controller's
 * stance-QP force block, main.cpp:1471-1647): for QP q, feet = foot positions
 * relative to the CoM (tiled, nv = 12: BR, BL, FL, FR, x y z each) and wrench =
 * desired wrench W (nv = 6); stance = bitmask of the feet in contact (bit i =
 * foot i), mu = friction coefficient.  Writes the plan's tiled inputs
 *   P = 50 Jc Jc' + I,  c = -50 Jc W,  A = Jc',  b = W,  G = friction blocks,  h = 0
 * with Jc,i = [I3, -[r_i]x] (zero for a swing foot).  The plan must have the
 * pattern of such a QP (QPB_ESHAPE otherwise; checked without touching the GPU). */
int  qpb_assemble_contact(const qpb_plan *plan, long B, const double *feet, const double *wrench,
                          int stance, double mu, double *P, double *A, double *G,
                          double *c, double *h, double *b, void *stream);

/* On-device assembly of the controller's own stance QP 30/68/18 (SURVEY §8f row 3,
 * main.cpp:1471-1647) from the robot terms the controller reads each tick, for B
 * QPs into the plan's tiled inputs.  Robot terms, QPB_ROBOT_NV doubles per QP, in
 * this order: Jst[12][18] (JacCOM_lin, foot rows BR BL FL FR x [CoM 6 | joints 12],
 * row-major), Mcom[6][6] (MassMatrixCOM(0:6,0:6)), Mjj[12][12] (MassMatrixCOM(6:18,
 * 6:18)), bias[18] (BiasCOM), jdqd[12] (JdqdCOM_lin), wdes[6] (Wcom_des), q[12],
 * dq[12], qmin[12], qmax[12].  terms_shared = 1: one copy for every QP (one robot,
 * many candidate targets: then pass the per-candidate wrench in wdes, tiled nv = 6);
 * 0: tiled, nv = QPB_ROBOT_NV.  wdes NULL: the terms' own.  check (DEVICE, [B] ints,
 * or NULL): 1 when every entry of the QP outside the plan's pattern is exactly 0,
 * as the plan assumes (QP_SETUP_dense drops exact zeros), else 0.  The plan must be
 * 30/68/18 (QPB_ESHAPE otherwise). */
#define QPB_ROBOT_NV 480
int  qpb_assemble_controller(const qpb_plan *plan, long B, const double *terms, int terms_shared,
                             const double *wdes, double mu, double *P, double *A, double *G,
                             double *c, double *h, double *b, int *check, void *stream);

/* APF-sampled targets (main.cpp:1263-1422) -> the desired CoM wrench each candidate
 * QP tracks (main.cpp:1484-1571).  State of one tick (host struct, shared by all
 * candidates); targets: tiled nv = 2, the candidate target point (x, y) of the
 * attractive field; outputs tiled: wrench nv = 6 (Wcom_des), com_des nv = 6
 * (CoMPosDes, or NULL).  The TOWR spline between target and tick is out of scope:
 * CoMPosD = CoMPosDes, CoMVelD = 0. */
typedef struct qpb_apf_state {
    double ee[4][2];          /* foot positions (x, y): BR, BL, FL, FR (ee*pos)                */
    double com[6];            /* CoM pose: x y z roll pitch yaw                                 */
    double com_vel[6];        /* CoM twist                                                      */
    double acc_des[6];        /* CoMAccD                                                        */
    double des_orient[2];     /* des_com_pos[3], des_com_pos[4]                                 */
    double rob_foot[4];       /* robustness indices rob_foot_br, _bl, _fl, _fr                  */
    double versor[4][2];      /* repulsive-field directions br, bl, fl, fr (main.cpp:454-457)   */
    double lat_versor[2];
    double R_wb[9];           /* _world_H_base rotation, row-major                              */
    double Mcom[36];          /* MassMatrixCOM(0:6,0:6), row-major                              */
    double mass;              /* robot_mass                                                     */
    int rep_field, min_exit, fake_crawl;
} qpb_apf_state;
int  qpb_apf_wrench(long K, const qpb_apf_state *st, const double *targets, double *wrench,
                    double *com_des, void *stream);
/* The robustness state of one gait step, as the controller derives it before the
 * fields (main.cpp:1273-1321): every foot's index is smoothed,
 * rob_foot = 0.35 rob_foot + 0.65 h_prev / period_st (h_prev: the step's
 * accumulated 1 / foot height of BR, BL, FL, FR; period_st: the step's duration),
 * and fake_crawl = (mean of the four < 0.34).  Updates st in place (host, no GPU);
 * the mean (robf_to_mean) goes to *robf_mean when not NULL. */
int  qpb_apf_update(qpb_apf_state *st, const double h_prev[4], double period_st, double *robf_mean);

/* ---- the multi-GPU argmin gather: RCCL over xGMI ----
 * One process per GPU, each solving its own shard (no data-path collective).
 * A communicator is an ncclComm_t: the caller's own, or one made here from a
 * unique id (QPB_COMM_ID_BYTES) that rank 0 creates and every rank receives out
 * of band.  RCCL is loaded on first use (librccl.so.1). */
#define QPB_COMM_ID_BYTES 128
int  qpb_comm_get_unique_id(void *id /* QPB_COMM_ID_BYTES */);
int  qpb_comm_init(void **comm, int nranks, const void *id, int rank);   /* on the current HIP device */
void qpb_comm_destroy(void *comm);
/* Ranks RCCL reports for the communicator (ncclCommCount). */
int  qpb_comm_count(void *comm, int *nranks);
/* Every rank calls this after qpb_solve_best on its shard: best = that shard's
 * {fval, index} (DEVICE), x = its tiled x (nv = n, B QPs), base = global index of
 * its QP 0.  Builds the rank's payload {fval, base + index, x*[n]} on the device,
 * all-gathers the 16 + 8n bytes of every rank (ncclAllGather) and reduces them on
 * the device: out (DEVICE, 2 + n doubles) = {fval, global index, x*} of the
 * global winner (lowest fval among optimal QPs, ties -> lowest global index; none
 * -> {+inf, -1, NaN...}).  Stream-ordered on `stream`; replaces the per-candidate
 * selection the controller would otherwise do on the host. */
int  qpb_argmin_allgather(const double *best, const double *x, long n, long B, long base, void *comm,
                          double *out, void *stream);
/* Step 3 alone: out = winner over `world` gathered payloads of width 2 + n
 * (DEVICE pointers). */
int  qpb_argmin_reduce(const double *gathered, long world, long n, double *out, void *stream);

/* ---- plan groups: one launch for a batch of mixed sparsity patterns ----
 * The APF planner's candidates differ in their stance sets (gait phases), i.e.
 * in their KKT patterns (configs[2]).  A group fuses up to 16 row-form plans
 * (qpb_plan_info.wave_qpw == 4: n, p <= 16, m <= 32, e.g. every contact-force
 * pattern) into ONE kernel: member i's QPs run in their own blocks with exactly
 * the code of qpb_solve on that plan (bit-identical results), and with best
 * != NULL the argmin over the whole concatenated batch (member 0's QPs first,
 * then member 1's, ...) is reduced inside the same launch.  Replaces one
 * QP_SETUP_dense + QP_SOLVE per candidate (qpSWIFT.c:260-456, 473-644) for a
 * mixed batch.  The plans may be destroyed after qpb_group_create. */
typedef struct qpb_group qpb_group;
typedef struct qpb_io {          /* one member's batch: DEVICE pointers, tiled SoA as qpb_solve */
    long B;
    const double *P, *A, *G, *c, *h, *b;
    double *x, *y, *z, *s;
    int *flag, *iters;
    double *fval, *stats;        /* stats may be NULL */
} qpb_io;
int  qpb_group_create(qpb_group **group, qpb_plan *const *plans, int nplans);
void qpb_group_destroy(qpb_group *group);
long qpb_group_source(const qpb_group *group, char *buf, long cap);
int  qpb_group_compile(qpb_group *group);
/* io[nplans]; best: DEVICE {fval, global index} or NULL.  Asynchronous on stream. */
int  qpb_group_solve(qpb_group *group, const qpb_io *io, const qpb_settings *st, double *best, void *stream);

const char *qpb_last_error(void);
const char *qpb_version(void);
/* Identity (version text) of the compiler that builds the generated kernels:
 * ROCm's clang run as a child process (pinned, whatever HIP libraries the host
 * process loaded), or hiprtc + the comgr it resolved when clang is absent.  The
 * code-object cache is keyed by it. */
const char *qpb_compiler(void);
/* DPP hazard audit of a gfx950 code object (the check every generated kernel
 * with inline-asm DPP passes before it is cached): 1 clean, 0 a write of a DPP
 * instruction's VGPR operand within 2 wait states or a VALU EXEC write within 5
 * (report says where), -1 cannot audit (no llvm-objdump). */
int qpb_audit_dpp(const void *code, long size, char *report, long cap);
/* The assembly-level repair every generated kernel goes through (qpb_hazard.cpp
 * join_fixup): in the gfx950 assembly text (NUL-terminated, rewritten in place, at
 * most cap bytes including the NUL), move lane-masked instructions the register
 * allocator placed between a divergent region's skip target (s_cbranch_execz) and its
 * EXEC restore (s_or_b64 exec, exec, ..) to just after the restore.  Returns the number
 * of repaired joins, -k when k could not be repaired, QPB_EINVAL when the result does
 * not fit cap. */
long qpb_join_fixup(char *text, long cap, char *report, long rcap);
/* The drop-in's persistent solvers on the calling thread (include/qpSWIFT.h):
 * out[0] = device solves they answered, out[1] = kernel launches they took
 * (first use, relaunch after an idle exit or new arguments), out[2] / out[3] =
 * nanoseconds the resident wave spent on the last cold (setup) / warm (QP_SOLVE)
 * request, from seeing it to posting the answer (s_memrealtime). */
int qpb_dropin_serve_stats(long out[4]);
/* Post the stop word to the calling thread's queued persistent drop-in waves without
 * waiting (they leave within microseconds): call before a device-wide synchronisation
 * (hipDeviceSynchronize) in a thread that also ticks the drop-in, or it may wait out
 * QPSWIFT_HIP_SERVE_IDLE_MS.  qpb_solve / qpb_solve_best / qpb_solve_warm /
 * qpb_group_solve do this themselves.  The next QP_SOLVE relaunches (~20 us). */
int qpb_dropin_quiesce(void);
/* The persistent solver's effective settings for this process (read once from the
 * environment): idle_ms = QPSWIFT_HIP_SERVE_IDLE_MS (default 20), life_ms = the
 * multi-request lifetime -- 0 (one request per wave, the shipped mode) unless
 * QPSWIFT_HIP_SERVE_LIFE_MS > 0 AND QPB_SERVE_DIAG=1 (a diagnostics-only mode with an
 * open defect, DESIGN_HISTORY §7.5).  Needs no GPU. */
int qpb_serve_config(double *idle_ms, double *life_ms);

#ifdef __cplusplus
}
#endif
#endif
