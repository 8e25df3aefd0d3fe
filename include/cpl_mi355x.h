/*
 * cpl_mi355x.h — C-ABI of the MI355X-native batched NLP-callback engine for
 * CentroidalPlanner's IFOPT evaluation path.
 *
 * One "instance" is one CentroidalPlanner problem (reference: cpl::solver::CplProblem,
 * /root/reference/src/CplProblem.cpp:6-82).  A batch is B independent instances that share
 * one problem template (contact set, environment, weights, bounds) and differ in their
 * decision vector x (and optionally mass and environment kind).
 *
 * Layout contract (IFOPT order, reference CplProblem ctor):
 *   x  (n = 3+9N)  : [CoM(3) | for i in contact_names order: F_i(3) p_i(3) n_i(3)]
 *                    (/root/reference/src/CplProblem.cpp:17-34)
 *   g  (m)         : [statics(6) | for k in std::map (lexicographic) order:
 *                     env(1) normal(3) cone(2)]            m = 6+6N   (with environment)
 *                    [statics(6) | for k in map order: cone(2)]  m = 6+2N (no environment,
 *                     the CoMPlanner path)                 (/root/reference/src/CplProblem.cpp:37-75)
 *   jac (nnz)      : values of the RowMajor CSR Jacobian IFOPT hands to IPOPT, explicit zeros
 *                    kept, columns ascending within a row. nnz = 6+42N (env) / 6+27N (none).
 *   f, grad (n)    : cost value and dense cost gradient (IpoptAdapter::eval_f / eval_grad_f).
 * Batched buffers are instance-major: instance b's record starts at b*n (x, grad), b*m (g),
 * b*nnz (jac), b (f, mass, env_tag).
 *
 * Conventions: every function returns CPL_OK (0) or a CPL_ERR_* status; nothing throws across
 * this boundary.  The reference's std::invalid_argument / std::out_of_range / std::runtime_error
 * map to CPL_ERR_INVALID_ARGUMENT / CPL_ERR_OUT_OF_RANGE / CPL_ERR_RUNTIME; the message of the
 * last failure on the calling thread is available from cpl_last_error().
 * Device pointers are caller-owned HIP allocations; `stream` is a hipStream_t (NULL = default).
 */
#ifndef CPL_MI355X_H
#define CPL_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPL_ABI_VERSION 1
#define CPL_MAX_CONTACTS 32

/* environment kinds (reference: cpl::env::EnvironmentClass subclasses,
 * /root/reference/include/CentroidalPlanner/Environment/Environment.h:13-48) */
#define CPL_ENV_NONE 0          /* CoMPlanner path: FrictionCone only, mu from a private Ground */
#define CPL_ENV_GROUND 1        /* cpl::env::Ground       (/root/reference/src/Ground.cpp) */
#define CPL_ENV_SUPERQUADRIC 2  /* cpl::env::Superquadric (/root/reference/src/Superquadric.cpp) */
#define CPL_ENV_MIXED 3         /* per-instance tag array selects GROUND (1) / SUPERQUADRIC (2) */

#define CPL_OK 0
#define CPL_ERR_INVALID_ARGUMENT 1 /* reference: std::invalid_argument */
#define CPL_ERR_OUT_OF_RANGE 2     /* reference: std::out_of_range (std::map::at) */
#define CPL_ERR_RUNTIME 3          /* reference: std::runtime_error */
#define CPL_ERR_HIP 4              /* a HIP runtime call failed */
#define CPL_ERR_UNSUPPORTED 5

/* IFOPT's infinity for one-sided bounds (ifopt::inf = 1.0e20; BoundSmallerZero = [-inf, 0]) */
#define CPL_INF 1.0e20

/*
 * The shared problem template.  Plain data: fill it with cpl_desc_init() and the setters below
 * (which validate exactly like the reference setters), or directly.
 * Per-contact arrays are indexed by the contact's position in contact_names (vector order).
 */
typedef struct cpl_problem_desc {
  int32_t abi_version;  /* = CPL_ABI_VERSION */
  int32_t n_contacts;   /* N, 1..CPL_MAX_CONTACTS */
  int32_t env_kind;     /* CPL_ENV_* */
  int32_t reserved0;
  /* map_order[k] = vector index of the k-th contact in std::map<std::string,...> order.
   * reference: constraints are added in map order (src/CplProblem.cpp:42), variables in vector
   * order (src/CplProblem.cpp:21).  They differ e.g. for "contact10" < "contact2". */
  int32_t map_order[CPL_MAX_CONTACTS];

  double mass;        /* default robot mass when no per-instance mass array is given
                         (CentroidalStatics::SetMass, src/Constraints/CentroidalStatics.cpp:20) */
  double gravity[3];  /* (0,0,-9.81), src/Constraints/CentroidalStatics.cpp:15 */
  double wrench[6];   /* manipulation wrench, default 0 (src/Constraints/CentroidalStatics.cpp:12) */
  double mu;          /* friction coefficient, default 1.0 (Environment.h:46) */
  double ground_z;    /* Ground level, default 0 (src/Ground.cpp:7) */
  double sq_C[3];     /* Superquadric centre, default (0,0,10) (src/Superquadric.cpp:7) */
  double sq_R[3];     /* radii, default (10,10,10) */
  double sq_P[3];     /* curvatures, default (10,10,10) */

  double F_thr[CPL_MAX_CONTACTS]; /* FrictionCone force threshold, default 0 (FrictionCone.cpp:14) */

  /* cost (MinimizeCentroidalVariables, src/MinimizeCentroidalVariables.cpp:5-27) */
  double W_com;                       /* default 1 */
  double com_ref[3];                  /* default (0,0,1) */
  double W_p[CPL_MAX_CONTACTS];       /* default 1 */
  double W_F[CPL_MAX_CONTACTS];       /* default 1 */
  double p_ref[CPL_MAX_CONTACTS][3];  /* default 0 */
  double F_ref[CPL_MAX_CONTACTS][3];  /* default 0 */

  /* variable bounds (Variable3D, src/Variable3D.cpp:12-13: default [-1000, 1000]) */
  double com_lb[3], com_ub[3];
  double F_lb[CPL_MAX_CONTACTS][3], F_ub[CPL_MAX_CONTACTS][3];
  double p_lb[CPL_MAX_CONTACTS][3], p_ub[CPL_MAX_CONTACTS][3];
  double n_lb[CPL_MAX_CONTACTS][3], n_ub[CPL_MAX_CONTACTS][3];
} cpl_problem_desc;

/* ---- library / diagnostics ------------------------------------------------------------ */
int32_t cpl_abi_version(void);
size_t cpl_desc_sizeof(void);          /* sizeof(cpl_problem_desc), for FFI layout checks */
const char* cpl_last_error(void);      /* message of the last failing call on this thread */
const char* cpl_status_string(int32_t status);

/* ---- problem template (host only) ----------------------------------------------------- */
/* Defaults of the reference constructors for N contacts named "contact1".."contactN"
 * (map order computed from those names).  Replaces CplProblem::CplProblem
 * (src/CplProblem.cpp:6-82) + CentroidalPlanner ctor mass check (src/CentroidalPlanner.cpp:12-15). */
int32_t cpl_desc_init(cpl_problem_desc* d, int32_t n_contacts, int32_t env_kind, double mass);
/* Recompute map_order from the contact names (vector order).  Duplicate or empty names are
 * rejected (the reference would silently alias them in its std::map). */
int32_t cpl_desc_set_contact_names(cpl_problem_desc* d, const char* const* names, int32_t n);
/* Validating setters (same checks as the reference):
 *   EnvironmentClass::SetMu        include/CentroidalPlanner/Environment/Environment.h:19-26
 *   Superquadric::SetParameters    src/Superquadric.cpp:12-29
 *   Variable3D::SetBounds          src/Variable3D.cpp:28-40  (var: 0=CoM,1=F,2=p,3=n) */
int32_t cpl_desc_set_mu(cpl_problem_desc* d, double mu);
int32_t cpl_desc_set_superquadric(cpl_problem_desc* d, const double C[3], const double R[3],
                                  const double P[3]);
int32_t cpl_desc_set_bounds(cpl_problem_desc* d, int32_t var, int32_t contact,
                            const double lb[3], const double ub[3]);

/* IpoptAdapter::get_nlp_info [IFOPT-ext]: n, m, nnz_jac_g. */
int32_t cpl_dims(const cpl_problem_desc* d, int32_t* n, int32_t* m, int32_t* nnz);
/* IpoptAdapter::eval_jac_g(values == NULL) [IFOPT-ext]: (iRow, jCol) of every stored entry in
 * RowMajor-CSR order.  Either pointer may be NULL.  Additionally `row_ptr` (m+1, may be NULL). */
int32_t cpl_structure(const cpl_problem_desc* d, int32_t* iRow, int32_t* jCol, int32_t* row_ptr);
/* IpoptAdapter::get_bounds_info [IFOPT-ext] over Variable3D::GetBounds (src/Variable3D.cpp:54-65)
 * and the ConstraintSet GetBounds overrides (CentroidalStatics.cpp:64-73, FrictionCone.cpp:48-58,
 * EnvironmentConstraint.cpp:31-40, EnvironmentNormal.cpp:36-50).  Any pointer may be NULL. */
int32_t cpl_bounds(const cpl_problem_desc* d, double* x_l, double* x_u, double* g_l, double* g_u);

/* ---- the hot path (device) ------------------------------------------------------------ */
/*
 * Evaluate `batch` instances in one launch.  Replaces, per instance, IpoptAdapter::eval_g,
 * eval_jac_g(values != NULL), eval_f and eval_grad_f [IFOPT-ext], i.e. the IFOPT walk over
 *   CentroidalStatics::GetValues / FillJacobianBlock  src/Constraints/CentroidalStatics.cpp:37-137
 *   EnvironmentConstraint::GetValues / FillJacobianBlock src/Constraints/EnvironmentConstraint.cpp:16-61
 *   EnvironmentNormal::GetValues / FillJacobianBlock  src/Constraints/EnvironmentNormal.cpp:16-87
 *   FrictionCone::GetValues / FillJacobianBlock       src/Constraints/FrictionCone.cpp:30-103
 *   MinimizeCentroidalVariables::GetCost / FillJacobianBlock src/MinimizeCentroidalVariables.cpp:124-192
 * and the Ground / Superquadric environment functions they call.
 *   d_x       [batch*n]   device, required
 *   d_mass    [batch]     device or NULL (then d->mass for every instance)
 *   d_env_tag [batch]     device uint8 (CPL_ENV_GROUND / CPL_ENV_SUPERQUADRIC); required iff
 *                         env_kind == CPL_ENV_MIXED, ignored otherwise
 *   d_g [batch*m], d_jac [batch*nnz], d_f [batch], d_grad [batch*n]: device outputs, any may be
 *   NULL (that output is skipped).
 * Asynchronous on `stream`; returns after the launch is enqueued.
 */
int32_t cpl_eval_batch(const cpl_problem_desc* d, int64_t batch, const double* d_x,
                       const double* d_mass, const uint8_t* d_env_tag, double* d_g,
                       double* d_jac, double* d_f, double* d_grad, void* stream);

/*
 * Per-shard residual norms of g against the constraint bounds (the per-shard figure the
 * multi-GPU path all-gathers): d_out[0] = max_b max_r viol(b,r), d_out[1] = sum_b sum_r viol^2,
 * where viol = max(g_l - g, g - g_u, 0) and NaN counts as +inf.  d_g is [batch*m] from
 * cpl_eval_batch.  Device output, 2 doubles.  Asynchronous on `stream`.
 */
int32_t cpl_residual_norms(const cpl_problem_desc* d, int64_t batch, const double* d_g,
                           double* d_out, void* stream);

/*
 * cpl_eval_batch and cpl_residual_norms of the g it produces, fused: each workgroup reduces the
 * violations of its tiles from the tile images in LDS (no second pass over g in HBM) and a
 * one-workgroup reduction launched right after on the same stream finishes the pair
 * (deterministic for a given device).  d_g is required; d_norms: device, 2 doubles, same
 * meaning as cpl_residual_norms.  Launches on different streams use separate workspaces.
 */
int32_t cpl_eval_batch_norms(const cpl_problem_desc* d, int64_t batch, const double* d_x,
                             const double* d_mass, const uint8_t* d_env_tag, double* d_g,
                             double* d_jac, double* d_f, double* d_grad, double* d_norms,
                             void* stream);

/*
 * Output layout flags of cpl_eval_batch_ex (bitwise OR; 0 = exactly cpl_eval_batch's layout):
 *   CPL_EVAL_JAC_FOLDED  values-only Jacobian records: the structurally constant entries (the same
 *     for every x) are skipped and the remaining ones keep IFOPT's RowMajor-CSR order.  Record
 *     length nnz_folded and the positions / values of the skipped entries: cpl_jac_fold_info().
 *     Ground (N contacts): 6 + 24N values (18 of every 42 per-contact entries are constants: the
 *     force-balance I3, src/Constraints/CentroidalStatics.cpp:93-95; the gradient (0,0,1),
 *     src/Ground.cpp:30-35; the zero normal Jacobian, src/Ground.cpp:46-50; the normal rows' n_r
 *     ones, src/Constraints/EnvironmentNormal.cpp:63-70).  Superquadric / mixed: 6 + 36N (the I3
 *     blocks and the ones).  No environment: 6 + 24N (the I3 blocks).
 *   CPL_EVAL_SOA  entry-major outputs: g [m][batch], jac [nnz(_folded)][batch], grad [n][batch]
 *     (f stays [batch]); the inputs stay instance-major.
 * Replaces nothing in the reference (IFOPT hands IPOPT the full CSR values, src/CentroidalPlanner.cpp:29
 * [IFOPT-ext]); for GPU-side consumers of the batch (the solve loop, a batched factorisation).
 */
#define CPL_EVAL_JAC_FOLDED 1
#define CPL_EVAL_SOA 2

int32_t cpl_eval_batch_ex(const cpl_problem_desc* d, int64_t batch, const double* d_x,
                          const double* d_mass, const uint8_t* d_env_tag, double* d_g,
                          double* d_jac, double* d_f, double* d_grad, double* d_norms,
                          int32_t flags, void* stream);

/*
 * The folded Jacobian layout of `d` (host only): *nnz_folded values per record; var_k[j] = the
 * CSR position (0..nnz-1, cpl_structure order) of folded value j; const_k[c] / const_val[c] = the
 * CSR position and value of skipped constant c, *n_const of them (nnz = nnz_folded + n_const).
 * Any pointer may be NULL.  Scattering the folded values to var_k and const_val to const_k gives
 * cpl_eval_batch's CSR values bit for bit.
 */
int32_t cpl_jac_fold_info(const cpl_problem_desc* d, int32_t* nnz_folded, int32_t* var_k,
                          int32_t* n_const, int32_t* const_k, double* const_val);

/* Kernel timing helper for the bench: launches the eval kernel of cpl_eval_batch (of
 * cpl_eval_batch_norms, i.e. with the fused per-workgroup norms, when d_norms != NULL) `reps` times
 * back to back on `stream` between two HIP events recorded on that same stream and returns the mean
 * milliseconds per eval kernel in *ms_per_launch.  The one-workgroup norms finish is not part of the
 * timed launches; one more complete launch afterwards leaves d_norms valid.  Synchronises the stream. */
int32_t cpl_time_eval_batch(const cpl_problem_desc* d, int64_t batch, const double* d_x,
                            const double* d_mass, const uint8_t* d_env_tag, double* d_g,
                            double* d_jac, double* d_f, double* d_grad, double* d_norms,
                            void* stream, int32_t reps, double* ms_per_launch);
/* the same for cpl_eval_batch_ex's layouts */
int32_t cpl_time_eval_batch_ex(const cpl_problem_desc* d, int64_t batch, const double* d_x,
                               const double* d_mass, const uint8_t* d_env_tag, double* d_g,
                               double* d_jac, double* d_f, double* d_grad, double* d_norms,
                               int32_t flags, void* stream, int32_t reps, double* ms_per_launch);

/* Tuning knobs (process-wide, for A/B measurements): kernel_variant 0 = auto (default: the
 * pipelined kernel for none/Ground, the tile-stationary kernel for Superquadric/mixed),
 * 1 = row-staged lane-per-instance, 2 = pipelined (persistent, warp-specialized), 3 =
 * tile-stationary, 4 = tile-stationary with the Jacobian written straight to the records, 5 =
 * entry-parallel (none / Ground, IFOPT CSR instance-major records: every g / jac entry computed by
 * the thread that stores it, no output image in LDS), 6 / 7 = mixed batches split by kind (the
 * Superquadric half LDS-staged on the contiguous kernel's uniform-axis tiles / Jacobian-direct; the
 * default for mixed is 6's form since round 6, 7's before);
 * tile_lds_kb = LDS budget of one workgroup (8..160 KiB; 0 = per-kernel
 * default: 48 KiB for both: the largest power-of-two tile that fits, e.g. 8 instances of 8
 * Superquadric contacts, 4 of 16); wg_threads = 128 or 256 for the tile kernel (default 256);
 * nt_stores = non-temporal output stores (default 1); ablate = measurement-only ablation
 * (0 = off, 1 = skip the compute phase, 2 = skip the output stores: results are then garbage; for
 * the kind split, bits 4 = its halves one after the other on one stream, 8 = the Ground half issued
 * first, 16 / 64 / 128 = the Ground list at 48 / 36 / 32 KiB instead of 40, 32 = the Superquadric tiles
 * at 40 KiB instead of 48, 256 / 512 = every Ground workgroup walking the tiles / two per CU instead of
 * one per CU while the Superquadric list is non-empty, 1024 / 2048 = the Ground half's compute waves at
 * wave priority 1 / 2, 4096 = the 4-instance Superquadric list tiles' gather / copy-out at the default
 * priority, 16384 = the Superquadric grid for half the batch (correct only when at most half the
 * instances are Superquadric); for the tile kernel, 8192 = its phase barriers skipped: garbage results).
 * Every variant computes bit-identical results.  Not thread-safe against concurrent launches. */
int32_t cpl_set_tuning(int32_t kernel_variant, int32_t tile_lds_kb, int32_t wg_threads, int32_t nt_stores,
                       int32_t ablate);

/* ---- host-buffer entry points ------------------------------------------------------------ */
/*
 * cpl_eval_batch_ex on HOST arrays (SURVEY.md §8(b) cpl_eval_batch_host): the same arguments and
 * layouts with host pointers, on a library-owned stream (one per device, serialised by a lock); the
 * call returns when the outputs are back in host memory.  Batches whose inputs + outputs fit 1 MiB
 * (the single-instance callback path) are copied into library-owned pinned host memory that the
 * kernel reads and writes directly (one launch, no DMA transfers); larger ones are staged through a
 * library-owned device workspace (grown on demand) with DMA copies.  The computation is the GPU kernel of cpl_eval_batch —
 * the library has no CPU evaluator.  This is what a single-instance IPOPT TNLP adapter binds
 * (IpoptAdapter::eval_g / eval_jac_g / eval_f / eval_grad_f behind src/CentroidalPlanner.cpp:29
 * [IFOPT-ext] hand host arrays); h_norms, if not NULL, receives the 2 residual norms.
 */
int32_t cpl_eval_batch_host(const cpl_problem_desc* d, int64_t batch, const double* h_x,
                            const double* h_mass, const uint8_t* h_env_tag, double* h_g,
                            double* h_jac, double* h_f, double* h_grad, double* h_norms,
                            int32_t flags);

/*
 * IPOPT's first-order derivative checker (option derivative_test = "first-order", which
 * src/CentroidalPlanner.cpp:26 sets for every solve [IPOPT-ext: TNLPAdapter::CheckDerivatives]),
 * batched: at every instance's x, each variable j is perturbed by h_j = perturbation * max(1, |x_j|)
 * and the forward differences (g(x + h_j e_j) - g(x)) / h_j and (f(x + h_j e_j) - f(x)) / h_j are
 * compared with the Jacobian column j (0 outside the structure) and grad f; an entry is flagged when
 *     |approx - exact| / max(|approx|, tol) > tol.
 * All batch * n perturbed points of a chunk are evaluated in one cpl_eval_batch launch.  IPOPT's
 * defaults: perturbation 1e-8, tol 1e-4 (IPOPT also moves the start point by a random
 * point_perturbation_radius first; here the check runs at the given x).
 *   d_x [batch*n], d_mass [batch] or NULL, d_env_tag [batch] (mixed only): device inputs
 *   d_inst_flagged [batch] int32 device or NULL: flagged entries per instance
 *   report: host, filled on return (the call synchronises `stream`)
 */
typedef struct cpl_derivative_report {
  int64_t n_checked;     /* entries compared: batch * n * (m + 1) */
  int64_t n_flagged;     /* entries above tol */
  double max_rel_error;  /* largest relative deviation over the batch */
  int64_t worst_instance;
  int32_t worst_row;     /* constraint row of the worst entry, -1 = objective gradient */
  int32_t worst_col;     /* variable */
  double worst_exact, worst_approx;
} cpl_derivative_report;

int32_t cpl_derivative_test(const cpl_problem_desc* d, int64_t batch, const double* d_x,
                            const double* d_mass, const uint8_t* d_env_tag, double perturbation,
                            double tol, int32_t* d_inst_flagged, cpl_derivative_report* report,
                            void* stream);

/* ---- the solve loop's Newton step (device) ------------------------------------------- */
/*
 * Batched primal-dual Newton step of the interior-point solve loop (centroidalplanner_amd/
 * batch_ipm.py; replaces, per instance, IPOPT's PDFullSpaceSolver / inertia-correcting
 * factorisation behind src/CentroidalPlanner.cpp:29 [IPOPT-ext]):
 *     [M  A^T] [dw]   [r1]
 *     [A   0 ] [dy] = [r2]        M = W + Sigma (nw x nw), A (m x nw), instance-major row-major
 * by the null-space method on a Householder QR of A^T, with IPOPT's inertia correction on the
 * device (delta_w on M until the reduced Hessian Z^T M Z is positive definite: first trial 1e-4 or
 * delta_w_last/3, growth x100 / x8; delta_c = 1e-8 mu^(1/4) |R|max on R's diagonal where A is
 * rank-deficient) and one step of iterative refinement.  One workgroup per instance; all of the
 * step's matrices in LDS.  nw <= 128, 0 <= m <= nw, and the LDS image must fit 160 KiB.
 *   mode 0: factorise + solve; d_mu [batch] (barrier parameter), d_delta_w_last [batch] or NULL,
 *           outputs d_delta_w, d_delta_c [batch], d_info [batch] (0 ok, 1 inertia not corrected)
 *   mode 1: re-solve with the factors mode 0 left in d_ws (second-order corrections: same M, A,
 *           r1 up to the caller, another r2)
 *   d_active [batch] uint8 or NULL: inactive instances are skipped (dw = dy = 0)
 *   d_ws: cpl_kkt_workspace_doubles(nw, m) doubles per instance (device)
 * Asynchronous on `stream`.
 */
int64_t cpl_kkt_workspace_doubles(int32_t nw, int32_t m);

/*
 * grad f + J^T y of every instance from the CSR Jacobian values of cpl_eval_batch (the Lagrangian
 * gradient the solve loop differentiates for its Hessian; IpoptAdapter has no such callback — IPOPT
 * forms it internally).  d_col_ptr [n+1], d_csc_k [nnz], d_csc_row [nnz]: the structure of
 * cpl_structure transposed (column j's entries are CSR positions d_csc_k[col_ptr[j]..col_ptr[j+1])
 * in rows d_csc_row[...]).  Instance b uses d_y[b / y_repeat].  NaN Jacobian values count as 0.
 */
int32_t cpl_lagrangian_grad(int64_t batch, int32_t n, int32_t m, int32_t nnz, const int32_t* d_col_ptr,
                            const int32_t* d_csc_k, const int32_t* d_csc_row, const double* d_grad,
                            const double* d_jac, const double* d_y, int32_t y_repeat, double* d_out, void* stream);
/*
 * cpl_eval_lagrangian_grad: grad f + J^T y of every instance straight from the eval kernel's LDS
 * tile image (the Jacobian never goes to HBM); bitwise the result of cpl_eval_batch (jac, grad)
 * followed by cpl_lagrangian_grad.  d_active (optional, one byte per y row): instances whose
 * y row is inactive are skipped (their output rows are left unwritten).  Pipelined path only
 * (Ground / no environment): returns CPL_ERR_UNSUPPORTED for Superquadric / mixed batches, whose
 * callers take the two-launch path.
 */
int32_t cpl_eval_lagrangian_grad(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                                 const uint8_t* d_env_tag, const int32_t* d_col_ptr, const int32_t* d_csc_k,
                                 const int32_t* d_csc_row, const double* d_y, int32_t y_repeat,
                                 const uint8_t* d_active, double* d_out, void* stream);
/*
 * cpl_lagrangian_hessian: the exact Hessian of f + y^T g over the free variables, [batch, nf, nf]
 * (d_free_idx: free variable -> column of x, int32), per instance (y: [batch, m]); instances with
 * d_active[b] == 0 are skipped.  Ground / no-environment problems only (their environment and
 * normal rows are linear): CPL_ERR_UNSUPPORTED otherwise.  Where a cone's tangential force is
 * exactly zero the |F_t| terms count as 0 (the reference's Jacobian is 0/0 there).
 */
int32_t cpl_lagrangian_hessian(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_y,
                               const uint8_t* d_active, const int32_t* d_free_idx, int32_t nf, double* d_H,
                               void* stream);
int32_t cpl_kkt_solve(int32_t mode, int64_t batch, int32_t nw, int32_t m, const double* d_M, const double* d_A,
                      const double* d_r1, const double* d_r2, const double* d_mu, const double* d_delta_w_last,
                      const uint8_t* d_active, double* d_dw, double* d_dy, double* d_delta_w, double* d_delta_c,
                      int32_t* d_info, double* d_ws, void* stream);
/*
 * The restoration phase's Newton system with p and n eliminated (IPOPT's restoration problem, as
 * its AugRestoSystemSolver reduces it; no reference counterpart — IPOPT's work behind
 * src/CentroidalPlanner.cpp:29): per instance
 *     [ W   A^T ] [dw]   [r1]     W [nw, nw] symmetric, A [m, nw], D = 1 / d_Dinv > 0 (diagonal)
 *     [ A   -D  ] [dy] = [r2]
 * through K = W + A^T D^-1 A with IPOPT's inertia correction (K + dW I positive definite; first
 * dW 1e-4 or d_delta_w_last / 3, growth x100 / x8): dw = K^-1 (r1 + A^T D^-1 r2), dy = D^-1 (A dw - r2).
 * d_delta_w_last is updated in place (the correction used); d_ws: nw * nw doubles per instance.
 * d_active [batch] uint8 or NULL: inactive instances are skipped.  0 <= m <= nw <= 128, and the LDS
 * image of nw^2 + nw + 2 max(m, 1) + m nw doubles must fit 160 KiB (nw = 128 holds m <= 30; nw = 47,
 * the 4-contact size, any m <= nw); larger systems return CPL_ERR_UNSUPPORTED before any launch.
 */
int32_t cpl_kkt_qd_solve(int64_t batch, int32_t nw, int32_t m, const double* d_W, const double* d_A,
                         const double* d_Dinv, const double* d_r1, const double* d_r2, const uint8_t* d_active,
                         double* d_delta_w_last, double* d_dw, double* d_dy, double* d_delta_w, double* d_ws,
                         void* stream);

/*
 * Solve-loop line search, fused per instance (csrc/cpl_ipm.hip; no reference counterpart — the
 * work IPOPT's BacktrackingLineSearch / FilterLSAcceptor do for one instance per trial, batched):
 *
 * cpl_ipm_trial_point: w_t = w + alpha[b] d (written to d_wt [batch, nw]) and the evaluation point
 *   X [batch, n]: X[b, free[k]] = mask[b] ? w_t[k] : w_keep[b, k] (k < nf), X[b, fixed[j]] =
 *   Xbase[b, fixed[j]].  Index arrays are int64, masks one byte per instance.
 * cpl_ipm_judge_take: IPOPT's acceptance test at the trial points (theta = sum |c|, barrier
 *   objective phi, filter of `nfilt` (theta, phi) entries per instance, switching condition /
 *   Armijo / sufficient decrease, theta_max); instances with searching & extra_mask (NULL: all)
 *   that pass copy (f_t, g_t, w_t, alpha, augment flag) into the line-search state and clear
 *   searching.  d_th_out / d_ok_out get theta and the test result of every instance.  mode 0: the
 *   filter test; 1: the feasibility step's test (theta cut by 10 %); 2: take unconditionally.
 *   row_slack[r] = slack index of inequality row r, -1 for an equality row.
 */
int32_t cpl_ipm_trial_point(int64_t batch, int32_t n, int32_t nf, int32_t nw, const int64_t* d_free_idx,
                            const int64_t* d_fixed_idx, const double* d_Xbase, const double* d_w, const double* d_dir,
                            const double* d_alpha, const uint8_t* d_mask, const double* d_w_keep, double* d_wt,
                            double* d_X, void* stream);
int32_t cpl_ipm_judge_take(int64_t batch, int32_t nw, int32_t m, int32_t nf, int32_t nfilt, const int32_t* d_row_slack,
                           const double* d_gl, const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0,
                           const double* d_wu0, const double* d_wt, const double* d_f_t, const double* d_g_t,
                           const double* d_alpha, const double* d_mu, const double* d_theta_k, const double* d_phi_k,
                           const double* d_gd, const uint8_t* d_switch_ok, const double* d_theta_max,
                           const double* d_filt_t, const double* d_filt_p, const uint8_t* d_extra_mask,
                           uint8_t* d_searching, double* d_st_f, double* d_st_g, double* d_st_w, double* d_st_alpha,
                           uint8_t* d_st_aug, double* d_th_out, uint8_t* d_ok_out, int32_t mode, void* stream);
/*
 * cpl_ipm_optimality: IPOPT's scaled optimality error (s_max = 100) at the current iterates, the
 *   convergence test (tol; acc_tol for acc_iter consecutive iterations) and the monotone barrier
 *   update (two rounds of mu <- max(min(0.2 mu, mu^1.5), tol/10) while err_mu <= 10 mu), each
 *   update resetting the instance's filter.  d_active / d_status (0 optimal, 1 acceptable) /
 *   d_acc are updated in place; d_d_inf, d_err0, d_base (max(|dual|/s_d, |c|)), the new mu and
 *   filter go to the *_out buffers.  nw <= 128.
 * cpl_ipm_max_step: the fraction-to-the-boundary step: primal (d_v2 = NULL) against the bounds
 *   d_lo (where d_hasL) / d_up (where d_hasU), or dual (multipliers d_v on d_hasL, d_v2 on d_hasU,
 *   kept positive); alpha <= 1 per instance, tau per instance.
 */
int32_t cpl_ipm_optimality(int64_t batch, int32_t nw, int32_t m, int32_t nfilt, int32_t nbounds, double tol,
                           double acc_tol, int32_t acc_iter, const double* d_A, const double* d_gw, const double* d_c,
                           const double* d_w, const double* d_y, const double* d_zL, const double* d_zU,
                           const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                           const double* d_mu, const double* d_filt_t, const double* d_filt_p,
                           const int64_t* d_fcount, uint8_t* d_active, int64_t* d_status, int64_t* d_acc,
                           double* d_d_inf, double* d_err0, double* d_base, double* d_mu_out, double* d_filt_t_out,
                           double* d_filt_p_out, int64_t* d_fcount_out, void* stream);
int32_t cpl_ipm_max_step(int64_t batch, int32_t nw, const double* d_v, const double* d_dir, const double* d_v2,
                         const double* d_dir2, const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_lo,
                         const double* d_up, const double* d_tau, double* d_out, void* stream);
/*
 * cpl_ipm_newton_setup: Sigma, grad_phi, r1 = -(grad_phi + A^T y), r2 = -c, M = diag(Sigma) + the
 *   nf x nf Hessian block d_H (NULL: none; h_sym: d_H is the raw central-difference matrix and
 *   0.5 (H + H^T) is added) — theta = |c|_1, the barrier objective phi and the feasibility step's diagonal
 *   Sigma + sqrt(mu) / max(1, |w|)^2, per instance.
 * cpl_ipm_fd_points: the 2 nf central-difference points x +- h e_k of every instance
 *   (h = fd_step max(|x_k|, 1); freepos[col] = free index of a column or -1) and the steps.
 * cpl_ipm_fd_hessian_raw: (gL[k, free j] - gL[nf + k, free j]) / (2 h_k) from the Lagrangian
 *   gradients at those points, [batch, nf, nf].
 * cpl_ipm_post_step: dzL, dzU from the primal step, the primal and dual fraction-to-the-boundary
 *   steps, gd = grad_phi . dw, the switching-condition flags (bit 0: gd < 0, bit 1: theta <= theta_min;
 *   the judge's Armijo branch needs both, its filter-augmentation test IPOPT's IsFtype, bit 0 alone),
 *   delta_w_last on active instances.
 * cpl_ipm_accept: filter augmentation / reset, y, z (kappa_Sigma safeguard), w, mu and iteration
 *   counters written back in place (d_failed: filter reset rows, d_rest: rows keeping z; both optional).
 * cpl_ipm_masked_rows: dst[b, :] = src[b, :] where mask[b].
 * d_active (optional, where present): instances with active[b] == 0 are skipped — their outputs
 * are left unwritten (converged instances of the solve loop, whose Newton data is never read).
 */
int32_t cpl_ipm_newton_setup(int64_t batch, int32_t nw, int32_t m, int32_t nf, const double* d_w, const double* d_zL,
                             const double* d_zU, const double* d_gw, const double* d_A, const double* d_y,
                             const double* d_c, const double* d_f, const double* d_mu, const uint8_t* d_hasL,
                             const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0, const double* d_H,
                             int32_t h_sym, double* d_M, double* d_r1, double* d_r2, double* d_gphi, double* d_mr_diag,
                             double* d_theta, double* d_phi, const uint8_t* d_active, void* stream);
int32_t cpl_ipm_fd_hessian_raw(int64_t batch, int32_t n, int32_t nf, const int64_t* d_free_idx, const double* d_gL,
                               const double* d_h, double* d_H, const uint8_t* d_active, void* stream);
int32_t cpl_ipm_fd_points(int64_t batch, int32_t n, int32_t nf, double fd_step, const int32_t* d_freepos,
                          const double* d_X, double* d_Xp, double* d_h, const uint8_t* d_active, void* stream);
int32_t cpl_ipm_post_step(int64_t batch, int32_t nw, const double* d_w, const double* d_dw, const double* d_zL,
                          const double* d_zU, const double* d_gphi, const double* d_mu, const double* d_tau,
                          const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                          const double* d_theta, const double* d_theta_min, const uint8_t* d_active,
                          const double* d_delta_w, double* d_dwl, double* d_dzL, double* d_dzU, double* d_a_max,
                          double* d_a_z, double* d_gd, uint8_t* d_switch_ok, void* stream);
int32_t cpl_ipm_accept(int64_t batch, int32_t nw, int32_t m, int32_t nfilt, const uint8_t* d_active,
                       const uint8_t* d_aug, const uint8_t* d_failed, const uint8_t* d_rest, const double* d_alpha,
                       const double* d_a_z, const double* d_theta, const double* d_phi, const double* d_filt_t_in,
                       const double* d_filt_p_in, const int64_t* d_fcount_in, const double* d_w_new,
                       const double* d_dy, const double* d_dzL, const double* d_dzU, const double* d_mu,
                       const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                       double* d_w, double* d_y, double* d_zL, double* d_zU, double* d_mu_state, int64_t* d_iters,
                       double* d_filt_t, double* d_filt_p, int64_t* d_fcount, void* stream);
int32_t cpl_ipm_masked_rows(int64_t batch, int64_t row_len, const uint8_t* d_mask, const double* d_src, double* d_dst,
                            void* stream);
/* cpl_ipm_dense_a: A = [J_free | -P] dense [batch, m, nw] from the Jacobian records of nnz values
 * (IFOPT CSR, or the folded layout of CPL_EVAL_JAC_FOLDED): amap[row, free column] = position in the
 * record, -1 for a structural zero (or a skipped constant 0), -2 for a skipped constant 1;
 * row_slack: slack of each inequality row or -1; NaN -> 0. */
int32_t cpl_ipm_dense_a(int64_t batch, int32_t m, int32_t nw, int32_t nf, int32_t nnz, const int32_t* d_amap,
                        const int32_t* d_row_slack, const double* d_jac, double* d_A, const uint8_t* d_active,
                        void* stream);

/* ---- the native batched solve engine (device) ------------------------------------------ */
/*
 * cpl_solver: many concurrent CentroidalPlanner solves in lock-step on one GPU — IPOPT's
 * primal-dual interior-point method (filter line search, second-order corrections, monotone barrier
 * update, inertia-correcting Newton steps) with every callback of every instance
 * one cpl_eval_batch launch, the Newton step in cpl_kkt_solve and the per-instance iteration work
 * in the cpl_ipm_* kernels; one iteration is captured once as a HIP graph and replayed with no host
 * synchronisation but a one-iteration-behind "any instance active" flag.  Replaces, per instance,
 * ifopt::IpoptSolver::Solve behind CentroidalPlanner::Solve (src/CentroidalPlanner.cpp:22-34).
 * Converged instances stay in the batch (frozen) until every instance has stopped.
 */
#define CPL_HESSIAN_EXACT 0          /* analytic Lagrangian Hessian (Ground / no environment), else FD */
#define CPL_HESSIAN_LIMITED_MEMORY 1 /* IPOPT's L-BFGS (6 pairs, scalar1): IFOPT's IpoptSolver default */
#define CPL_HESSIAN_FD 2             /* central differences of grad f + J^T y */

#define CPL_SOLVE_OPTIMAL 0
#define CPL_SOLVE_ACCEPTABLE 1
#define CPL_SOLVE_MAX_ITER 2
#define CPL_SOLVE_INFEASIBLE 3   /* restoration phase converged to a point of local infeasibility */
#define CPL_SOLVE_RESTO_FAILED 4 /* the restoration phase converged to a feasible point the original
                                    filter rejects, again after its tolerance was tightened (IPOPT's
                                    RESTORATION_CONVERGED_TO_FEASIBLE_POINT); a failed restoration line
                                    search resets p, n instead (RestoRestorationPhase); or the line search
                                    failed at an almost feasible point (theta <= 1e-2 tol), where IPOPT
                                    calls no restoration phase.  When an earlier regular iterate was at
                                    the acceptable level, that point is restored and the status is
                                    CPL_SOLVE_ACCEPTABLE instead (IPOPT's backup acceptable point) */

typedef struct cpl_solve_options {
  int32_t max_iter;        /* 3000 (IPOPT's default) */
  int32_t hessian;         /* CPL_HESSIAN_*, default CPL_HESSIAN_EXACT */
  int32_t max_ls;          /* backtracking trials per iteration at most (also alpha_min), 40 */
  int32_t max_soc;         /* second-order corrections on the first trial, 4 (IPOPT max_soc) */
  int32_t acceptable_iter; /* 15 */
  int32_t use_graph;       /* capture the iteration as a HIP graph, 1 */
  int32_t compact;         /* active-set compaction, 1: once at most half of the batch is still
                              active, the active instances move to the front and the lock-step
                              batch shrinks to them (halvings of the size, >= 256 rows; one graph per
                              size); the results come back in the instances' own order */
  int32_t ls_kernel;       /* the first line-search trial, its second-order corrections and the
                              backtracking in ONE launch (systems the one-wave KKT kernel factorises:
                              nw = 47, m = 30): 2 (default) at every batch size, 1 for lock-step
                              batches of at most 256 rows, 0 never (one launch per step of the first
                              trial) — the same iterates bit for bit either way */
  double tol;              /* 1e-8 */
  double acceptable_tol;   /* 1e-6 */
  double mu_init;          /* 0.1 */
  double fd_step;          /* 1e-6 (CPL_HESSIAN_FD / Superquadric exact) */
  double fallback_viol_tol; /* 0 (off, the default: IPOPT returns its last iterate).  Opt-in, not IPOPT:
                              > 0 — a solve that ends without convergence (max_iter, local infeasibility,
                              restoration failure) at an iterate whose original constraints are
                              violated by more than this returns the lowest-objective iterate it met
                              that satisfied them to this tolerance, when there was one (status
                              unchanged; cpl_solver_fallbacks says which instances).  Only x is
                              replaced: the multipliers and dual_inf of such an instance still belong
                              to its last iterate. */
  int32_t nlp_scaling;     /* 1 (default): IPOPT's gradient-based NLP scaling (nlp_scaling_method, which
                              IFOPT's IpoptSolver and the reference leave at its default,
                              src/CentroidalPlanner.cpp:26-27), computed once at the starting point:
                              df = max(1e-8, 100 / max|grad f|) when max|grad f| > 100; for each block
                              of rows (equalities; inequalities) whose largest row gradient exceeds 100,
                              dc_i = max(1e-8, 100 * (1 / max(100, max_j |J_ij|))) on each of its rows
                              (gradients over the free variables, a NaN entry counting as 0).  The
                              iteration and its tolerances run on the scaled problem; x is unscaled, the
                              returned multipliers are the unscaled ones (dc y / df).  0: no scaling. */
  int32_t jacobian_regularization; /* a rank-deficient constraint Jacobian (|R_jj| < 1e-10 |R|max in the QR
                              of A^T): 0 (default) — delta_c = 1e-8 mu^0.25 |R|max added to R's small
                              pivots (the three restatements' treatment); 1 — IPOPT's: the (2,2) block
                              [[W + dW I, A^T], [A, -delta_c I]], delta_c = 1e-8 mu^0.25
                              (jacobian_regularization_value / _exponent), solved as the augmented system
                              in (dw, s) with A~ = [A, -sqrt(delta_c) I] on the workgroup KKT kernel;
                              needs nw + m <= 128.  The restatements carry the same option
                              (oracle cplo_set_jac_reg, batch_ipm_solve(jacobian_regularization="ipopt")). */
} cpl_solve_options;

typedef struct cpl_solver cpl_solver;

void cpl_solve_options_default(cpl_solve_options* o);
/* A solver for `batch` instances of the template `d` (copied): plans the problem (free / fixed
 * variables, slacks, the Jacobian maps) and allocates every device buffer on the current device.
 * nw = free variables + inequality rows must be <= 128. */
int32_t cpl_solver_create(const cpl_problem_desc* d, int64_t batch, const cpl_solve_options* o, cpl_solver** out);
int32_t cpl_solver_destroy(cpl_solver* s);
/* Solve every instance from d_x0 [batch, n] (device; masses d_mass [batch] or NULL, tags
 * d_env_tag for mixed batches) on `stream`; returns when every instance has stopped.  Outputs
 * (device, any may be NULL): d_x [batch, n] (projected onto the original bounds, IPOPT
 * honor_original_bounds), d_y [batch, m] constraint multipliers, d_status (CPL_SOLVE_*), d_iters
 * (iterations per instance), d_obj (f at d_x), d_primal_inf (max violation at d_x), d_dual_inf (the
 * last iterate's dual infeasibility OF THE SCALED PROBLEM when nlp_scaling is on — IPOPT's scaled
 * quantity; d_y is returned unscaled, dc y / df).
 * *iterations_run (host, may be NULL): lock-step iterations of the batch; *evaluations: eval launches. */
int32_t cpl_solver_solve(cpl_solver* s, const double* d_x0, const double* d_mass, const uint8_t* d_env_tag,
                         double* d_x, double* d_y, int32_t* d_status, int32_t* d_iters, double* d_obj,
                         double* d_primal_inf, double* d_dual_inf, int32_t* iterations_run, int64_t* evaluations,
                         void* stream);
/* dims of the solver's primal-slack system: nf free variables, nI inequality rows (nw = nf + nI) */
int32_t cpl_solver_dims(const cpl_solver* s, int32_t* nf, int32_t* n_ineq, int32_t* graph_captured);
/* the last solve's active-set compactions and its final lock-step batch size */
int32_t cpl_solver_stats(const cpl_solver* s, int32_t* compactions, int64_t* final_rows);
/* the last solve's fallback flags per instance into d_out [batch] (device uint8): 1 = the returned x is
 * the best feasible iterate, not the last one (cpl_solve_options.fallback_viol_tol) */
int32_t cpl_solver_fallbacks(const cpl_solver* s, uint8_t* d_out, void* stream);
/* the last solve's restoration-phase entries per instance into d_out [batch] (device int64) */
int32_t cpl_solver_restorations(const cpl_solver* s, int64_t* d_out, void* stream);
/* the last solve's NaN constraint-Jacobian entries per instance at its start point (x0 with the fixed
 * variables at their values; the cone's 0/0 at F_t = 0, src/Constraints/FrictionCone.cpp:85-87), which
 * the iteration takes as 0 where IPOPT would receive NaN, into d_out [batch] (device int32) */
int32_t cpl_solver_nan_jacobian(const cpl_solver* s, int32_t* d_out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CPL_MI355X_H */
