/*
 * nfft4gp_amd.h -- C ABI of the MI355X-native NFFT additive-kernel operator.
 *
 * Drop-in replacement for the hot-path subset of the reference header
 *   INC/nfft4gp_headers.h:9-23  (aggregating INC/_linearalg.h, _solvers.h, _preconds.h, _external.h)
 * of Hitenze/Preconditioned_Additive_Gaussian_Processes_with_Fourier_Acceleration.
 *
 * Differences from the reference header, all deliberate:
 *  - no NFFT3/FFTW includes (INC/_external.h:4-20): str_adj is declared with fastsum_plan opaque;
 *  - vectors x, y, rhs may be HOST or DEVICE (hipMalloc) pointers; the library detects which with
 *    hipPointerGetAttributes.  Device pointers run with no PCIe traffic and no host sync, enqueued
 *    on the stream set by Nfft4GPAmdSetStream (default: the null stream, ordered with torch's
 *    default stream).  Host pointers are staged through device buffers and the call is synchronous.
 *  - every computation runs on the GPU; there is no CPU fallback.  If no HIP device is present the
 *    operator entry points print an error and return -1.
 *  - Nfft4GPSolverPcg keeps its vectors in HBM.  Callbacks of this library (the NFFT matvecs,
 *    Nfft4GPAmdNysSolve, Nfft4GPAmdFsaiSolve, Nfft4GPAmdAfnSolve) receive device pointers; any other callback -- e.g. the reference's own
 *    Nfft4GPDenseMatSymv -- is called with HOST vectors staged around the call, exactly as the
 *    reference calls it (see Nfft4GPAmdSetCallbackPointerMode).
 *
 * Precision: NFFT4GP_DOUBLE is double (the reference default, SRC/utils/utils.h:28-31).
 */
#ifndef NFFT4GP_AMD_H
#define NFFT4GP_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef NFFT4GP_DOUBLE
#define NFFT4GP_DOUBLE double
#endif

#ifndef NFFT4GP_KERNEL_MAX_PARAMS
#define NFFT4GP_KERNEL_MAX_PARAMS 5 /* SRC/linearalg/kernels.h:59-61 */
#endif

/* ---- function-pointer types (unchanged) ------------------------------------------------------ */
/* SRC/linearalg/kernels.h:49 */
typedef int (*func_kernel)(void *str, NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *permr, int kr,
                           int *permc, int kc, NFFT4GP_DOUBLE **Kp, NFFT4GP_DOUBLE **dKp);
/* SRC/solvers/solvers.h:21 */
typedef int (*func_solve)(void *precond, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
/* SRC/solvers/solvers.h:49 */
typedef int (*func_symmatvec)(void *matrix, int n, NFFT4GP_DOUBLE alpha, NFFT4GP_DOUBLE *x,
                              NFFT4GP_DOUBLE beta, NFFT4GP_DOUBLE *y);
/* SRC/utils/utils.h (func_free) */
typedef void (*func_free)(void *str);
/* SRC/solvers/solvers.h:58, :66, :79: preconditioner trace / logdet / dM/dtheta x (GP loss gradient) */
typedef int (*func_trace)(void *str, NFFT4GP_DOUBLE **tracesp);
typedef NFFT4GP_DOUBLE (*func_logdet)(void *str);
typedef int (*func_dvp)(void *str, int n, int *mask, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE **yp);
/* SRC/preconds/precond.h:39-47 */
typedef int (*precond_kernel_setup)(NFFT4GP_DOUBLE *data, int n, int ldim, int d, func_kernel fkernel,
                                    void *fkernel_params, int require_grad, void *precond_data);
/* SRC/optimizer/transform.h:15-20 */
typedef enum
{
   NFFT4GP_TRANSFORM_SOFTPLUS = 0,
   NFFT4GP_TRANSFORM_SIGMOID,
   NFFT4GP_TRANSFORM_EXP,
   NFFT4GP_TRANSFORM_IDENTITY
} nfft4gp_transform_type;

/* ---- kernel handle: field layout identical to SRC/linearalg/kernels.h:65-95 -------------------
 * Callers write _params[0] (f), _params[1] (l) and _noise_level (mu) directly
 * (SRC/optimizer/gp_loss.c:143-150, TESTS/TEST1/foo.cpp:222-224).  _external points at the
 * library's device-side plan (opaque). */
typedef struct NFFT4GP_KERNEL_STRUCT
{
   NFFT4GP_DOUBLE _params[NFFT4GP_KERNEL_MAX_PARAMS];
   int _iparams[NFFT4GP_KERNEL_MAX_PARAMS];
   int _max_n;
   int _omp;
   NFFT4GP_DOUBLE _noise_level;
   int _own_buffer;
   NFFT4GP_DOUBLE *_buffer;
   int _own_dbuffer;
   NFFT4GP_DOUBLE *_dbuffer;
   func_kernel _fkernel_buffer;
   int **_ibufferp;
   size_t *_libufferp;
   int _own_fkernel_buffer_params;
   void *_fkernel_buffer_params;
   size_t _ldwork;
   NFFT4GP_DOUBLE *_dwork;
   void *_external;
} nfft4gp_kernel, *pnfft4gp_kernel;

/* ---- per-component NFFT state: field layout identical to INC/_external.h:28-51 ----------------
 * Declared for source compatibility (a caller naming str_adj compiles).  NFFT3's fastsum_plan stays
 * opaque: no fastsum.h is needed, and the typedef below is the same one fastsum.h makes.  The
 * single-component handle's *Kp (Nfft4GPNFFTKernel{Gaussian,Matern12}Kernel) points at a str_adj that
 * holds the cached scalars of the reference (_kernel, _d, _sigma, _mu, _N, _p, _m, _eps, _n, _NN, _scale,
 * _kernel_scale); _x and the two plans are NULL: the centred points and the plans live in HBM. */
typedef struct fastsum_plan_ fastsum_plan;
typedef struct
{
   int _kernel; /* 0: Gauss, 1: Matern 1/2 */
   int _d;
   NFFT4GP_DOUBLE *_sigma;
   NFFT4GP_DOUBLE _mu;
   int _N;
   int _p;
   int _m;
   NFFT4GP_DOUBLE _eps;
   int _n;
   int _NN;
   NFFT4GP_DOUBLE *_x;
   NFFT4GP_DOUBLE _scale;
   NFFT4GP_DOUBLE _kernel_scale;
   fastsum_plan *_fastsum_original;
   fastsum_plan *_fastsum_derivative;
} str_adj, *pstr_adj;

/* ---- generic kernel parameter struct --------------------------------------------------------- */
/* replaces SRC/linearalg/kernels.c:404-436 */
void *Nfft4GPKernelParamCreate(int max_n, int omp);
/* replaces SRC/linearalg/kernels.c:438-470 */
void Nfft4GPKernelParamFree(void *str);

/* ---- NFFT single-component operator (INC/_external.h:60-200) ----------------------------------- */
/* replaces SRC/external/nfft_interface.c:3-42 */
void *Nfft4GPNFFTKernelParamCreate(int max_n, int dim);
/* replaces SRC/external/nfft_interface.c:44-77 */
void Nfft4GPNFFTKernelParamFree(void *kernel);
/* replaces SRC/external/nfft_interface.c:79-82 (no-op, used as func_free) */
void Nfft4GPNFFTKernelFree(void *str);
/* replaces SRC/external/nfft_interface.c:84-101 */
int Nfft4GPNFFTKernelParamFreeNFFTKernel(void *kernel);
/* replaces SRC/external/nfft_interface.c:103-127 */
int Nfft4GPNFFTKernelParamRemovePoints(void *kernel);
/* replaces SRC/external/nfft_interface.c:129-263 (func_kernel; *Kp = *dKp = component handle) */
int Nfft4GPNFFTKernelGaussianKernel(void *str, NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *permr, int kr,
                                    int *permc, int kc, NFFT4GP_DOUBLE **Kp, NFFT4GP_DOUBLE **dKp);
/* replaces SRC/external/nfft_interface.c:265-398 */
int Nfft4GPNFFTKernelMatern12Kernel(void *str, NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *permr, int kr,
                                    int *permc, int kc, NFFT4GP_DOUBLE **Kp, NFFT4GP_DOUBLE **dKp);
/* replaces SRC/external/nfft_interface.c:400-497 (func_symmatvec on the component handle) */
int Nfft4GPNFFTMatSymv(void *data, int n, NFFT4GP_DOUBLE alpha, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE beta,
                       NFFT4GP_DOUBLE *y);
/* replaces SRC/external/nfft_interface.c:499-620 (y is 3n: dK/df, dK/dl, dK/dmu) */
int Nfft4GPNFFTGradMatSymv(void *data, int n, NFFT4GP_DOUBLE alpha, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE beta,
                           NFFT4GP_DOUBLE *y);

/* ---- NFFT additive operator (the north-star path) ---------------------------------------------- */
/* replaces SRC/external/nfft_interface.c:622-674 */
void *Nfft4GPNFFTAdditiveKernelParamCreate(NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *windows, int nwindows,
                                           int dwindows);
/* replaces SRC/external/nfft_interface.c:676-734 (func_kernel; *Kp = *dKp = str) */
int Nfft4GPNFFTAdditiveKernelGaussianKernel(void *str, NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *permr,
                                            int kr, int *permc, int kc, NFFT4GP_DOUBLE **Kp, NFFT4GP_DOUBLE **dKp);
/* replaces SRC/external/nfft_interface.c:736-794 */
int Nfft4GPNFFTAdditiveKernelMatern12Kernel(void *str, NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *permr,
                                            int kr, int *permc, int kc, NFFT4GP_DOUBLE **Kp, NFFT4GP_DOUBLE **dKp);
/* replaces SRC/external/nfft_interface.c:796-817: y = beta*y + alpha*f^2*((1/nw) sum_c K_c + mu I) x */
int Nfft4GPAdditiveNFFTMatSymv(void *data, int n, NFFT4GP_DOUBLE alpha, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE beta,
                               NFFT4GP_DOUBLE *y);
/* replaces SRC/external/nfft_interface.c:819-840 */
int Nfft4GPAdditiveNFFTGradMatSymv(void *data, int n, NFFT4GP_DOUBLE alpha, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE beta,
                                   NFFT4GP_DOUBLE *y);
/* Nfft4GPAdditiveNFFTMatSymv on nrhs column-major device vectors X (ldx) -> Y (ldy): two vectors per pass
 * over the HBM layout (the layout read and the per-point decode shared).  The reference calls its matvec
 * once per vector (lanczos.c:490-574 probe by probe). */
int Nfft4GPAmdAdditiveMatSymvMulti(void *data, int n, int nrhs, NFFT4GP_DOUBLE alpha, const NFFT4GP_DOUBLE *X,
                                   long long ldx, NFFT4GP_DOUBLE beta, NFFT4GP_DOUBLE *Y, long long ldy);
/* replaces SRC/external/nfft_interface.c:842-856 */
void Nfft4GPAdditiveNFFTKernelFree(void *str);
/* replaces SRC/external/nfft_interface.c:873-1068: posterior mean at the n_predict points of data_all
 * (rows n..n+n_predict-1; vfkernel_data_l is a kernel handle over data_all) and, if std_predictp is not
 * NULL, the predictive standard deviation sqrt|K22_ii - K21_i K11^{-1} K12_i|.  *label_predictp /
 * *std_predictp: caller arrays (host or device) or NULL to get malloc'ed host arrays. */
int Nfft4GPAdditiveNFFTGpPredict(NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *data, NFFT4GP_DOUBLE *label, int n, int ldim,
                                 int d, NFFT4GP_DOUBLE *data_predict, int n_predict, int ldim_predict,
                                 NFFT4GP_DOUBLE *data_all, func_kernel fkernel, void *vfkernel_data,
                                 void *vfkernel_data_l, func_free kernel_data_free, func_symmatvec matvec,
                                 func_kernel precond_fkernel, void *precond_vfkernel_data,
                                 func_free precond_kernel_data_free, precond_kernel_setup precond_setup,
                                 func_solve precond_solve, void *precond_data, int atol, NFFT4GP_DOUBLE tol,
                                 int maxits, nfft4gp_transform_type transform, int print_level,
                                 NFFT4GP_DOUBLE *dwork, NFFT4GP_DOUBLE **label_predictp,
                                 NFFT4GP_DOUBLE **std_predictp);
/* replaces SRC/external/nfft_interface.c:858-871 (host memory, caller frees with free()) */
NFFT4GP_DOUBLE *Nfft4GPNFFTAppendData(NFFT4GP_DOUBLE *X1, int n1, int ldim1, int d, NFFT4GP_DOUBLE *X2, int n2,
                                      int ldim2);

/* ---- BLAS-1 vector ops (SRC/linearalg/vecops.c:3-155), host or device pointers ------------------ */
NFFT4GP_DOUBLE Nfft4GPVecNorm2(NFFT4GP_DOUBLE *x, int n);                       /* vecops.c:3-7 */
NFFT4GP_DOUBLE Nfft4GPVecDdot(NFFT4GP_DOUBLE *x, int n, NFFT4GP_DOUBLE *y);     /* vecops.c:9-13 */
void Nfft4GPVecFill(NFFT4GP_DOUBLE *x, size_t n, NFFT4GP_DOUBLE val);           /* vecops.c:47-69 */
void Nfft4GPVecScale(NFFT4GP_DOUBLE *x, size_t n, NFFT4GP_DOUBLE scale);        /* vecops.c:71-100 */
void Nfft4GPVecAxpy(NFFT4GP_DOUBLE alpha, NFFT4GP_DOUBLE *x, size_t n, NFFT4GP_DOUBLE *y); /* vecops.c:102-155 */
/* vecops.c:15-46: serial libc rand() / RAND_MAX (Rademacher: < 0.5 -> -1, else 1), as the reference */
void Nfft4GPVecRand(NFFT4GP_DOUBLE *x, int n);
void Nfft4GPVecRadamacher(NFFT4GP_DOUBLE *x, int n);

/* ---- PCG (SRC/solvers/pcg.c:3-206), device-resident ------------------------------------------- */
int Nfft4GPSolverPcg(void *mat_data, int n, func_symmatvec matvec, void *prec_data, func_solve precondfunc,
                     NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs, int maxits, int atol, NFFT4GP_DOUBLE tol,
                     NFFT4GP_DOUBLE *prel_res, NFFT4GP_DOUBLE **prel_res_v, int *piter, int print_level);

/* length of the rel_res_v array returned by the last Nfft4GPSolverPcg call on this process
 * (1 for the early exits of pcg.c:32-41 / :70-84, maxits+1 otherwise) */
int Nfft4GPAmdPcgHistoryLength(void);

/* ---- FGMRES, Lanczos, stochastic Lanczos quadrature, GP loss ------------------------------------
 * Same signatures and results as the reference; every n-vector lives in HBM, callbacks follow the PCG
 * rules above (this library's operators/preconditioners get device pointers, others host vectors).
 * prel_res_v / TDp / TEp are malloc'ed (free with free()). */
/* FGMRES's orthogonalisation: 0 (default) the reference's modified Gram-Schmidt (Nfft4GPModifiedGS,
 * matops.c:274-346: one launch per basis vector), 1 block classical Gram-Schmidt (two launches per pass
 * whatever the step; a second pass when the first drops ||w|| below 0.7071 of its value, the DGKS test of
 * matops.c:348-440; the same projections up to rounding; kdim <= 2046), 2 delayed CGS2 (the second pass
 * of column j run with step j + 1's first pass: two basis sweeps and one host read per step; with a
 * preconditioner the provisional directions z_j^0 = M^-1 v_j^0 are kept and x is updated through the delayed
 * pass's triangular recurrence).  The block modes restart from the true residual norm (fgmres.c:236-243
 * keeps the Givens estimate).  Env NFFT4GP_AMD_FGMRES_ORTHO.
 * Nfft4GPAmdFgmresSecondPasses: second passes taken since the last call (then reset). */
void Nfft4GPAmdSetFgmresOrtho(int ortho);
long long Nfft4GPAmdFgmresSecondPasses(void);
/* SRC/solvers/fgmres.c:3-252 (MGS without re-orthogonalisation; kdim <= 4094) */
int Nfft4GPSolverFgmres(void *mat_data, int n, func_symmatvec matvec, void *prec_data, func_solve precondfunc,
                        NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs, int kdim, int maxits, int atol, NFFT4GP_DOUBLE tol,
                        NFFT4GP_DOUBLE *prel_res, NFFT4GP_DOUBLE **prel_res_v, int *piter, int print_level);
/* SRC/solvers/lanczos.c:3-419 (preconditioned Lanczos, MGS2 re-orthogonalisation; maxits <= 4094) */
int Nfft4GPSolverLanczos(void *mat_data, int n, func_symmatvec matvec, void *prec_data, func_solve precondfunc,
                         NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs, int wsize, int maxits, int atol, NFFT4GP_DOUBLE tol,
                         NFFT4GP_DOUBLE *prel_res, NFFT4GP_DOUBLE **prel_res_v, int *piter, int *tsize,
                         NFFT4GP_DOUBLE **TDp, NFFT4GP_DOUBLE **TEp, int print_level);
/* SRC/solvers/lanczos.c:421-610: logdet(K)/n and its hyperparameter gradient; radamacher (n x nvecs,
 * host or device) or NULL for Nfft4GPVecRadamacher probes */
int Nfft4GPLanczosQuadratureLogdet(void *mat_data, void *dmat_data, int n, func_symmatvec matvec,
                                   func_symmatvec dmatvec, void *prec_data, func_solve precondfunc,
                                   func_trace tracefunc, func_logdet logdetfunc, func_dvp dvpfunc, int maxits,
                                   int nvecs, NFFT4GP_DOUBLE *radamacher, int print_level, NFFT4GP_DOUBLE *logdet,
                                   NFFT4GP_DOUBLE **dlogdetp);
/* SRC/optimizer/transform.c:4-89 */
int Nfft4GPTransform(nfft4gp_transform_type type, NFFT4GP_DOUBLE val, int inverse, NFFT4GP_DOUBLE *tvalp,
                     NFFT4GP_DOUBLE *dtvalp);
/* SRC/optimizer/gp_loss.c:96-307: loss = (y^T K^{-1} y + logdet K + log 2 pi) / (2n) and its gradient in
 * the transformed hyperparameters x = (f, l, mu) */
int Nfft4GPGpLoss(NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *data, NFFT4GP_DOUBLE *label, int n, int ldim, int d,
                  func_kernel fkernel, void *vfkernel_data, func_free kernel_data_free, func_symmatvec matvec,
                  func_symmatvec dmatvec, func_kernel precond_fkernel, void *precond_vfkernel_data,
                  func_free precond_vfkernel_data_free, precond_kernel_setup precond_setup, func_solve precond_solve,
                  func_trace precond_trace, func_logdet precond_logdet, func_dvp precond_dvp, func_free precond_reset,
                  void *precond_data, int atol, NFFT4GP_DOUBLE tol, int wsize, int maxits, int nvecs,
                  NFFT4GP_DOUBLE *radamacher, nfft4gp_transform_type transform, int *mask, int print_level,
                  NFFT4GP_DOUBLE *dwork, NFFT4GP_DOUBLE *loss, NFFT4GP_DOUBLE *grad);
/* how Nfft4GPSolverPcg hands vectors to its matvec / preconditioner callbacks:
 * -1 (default) device pointers for this library's own operators, host-staged vectors for any other
 *  function; 0 always host-staged; 1 always device pointers (for user callbacks written for HBM). */
void Nfft4GPAmdSetCallbackPointerMode(int mode);

/* ---- Nystrom ("RAN") preconditioner apply (SRC/preconds/nys.c:115-173) ----------------------------
 * The reference builds U (n x k), s, eta in Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660);
 * Nfft4GPAmdNysCreate takes those factors (host or device arrays) and keeps them in HBM with U's rows
 * already un-permuted, so the apply needs no gather. */
void *Nfft4GPAmdNysCreate(int n, int k, const NFFT4GP_DOUBLE *U, const NFFT4GP_DOUBLE *s, NFFT4GP_DOUBLE eta,
                          const int *perm);
/* same signature as Nfft4GPPrecondNysSolve (nys.c:115): x = M^{-1} rhs, func_solve */
int Nfft4GPAmdNysSolve(void *nys, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
void Nfft4GPAmdNysFree(void *nys);
/* Nystrom preconditioner SETUP on the GPU: Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660, require_grad
 * = 0) for the DENSE additive kernel (kernels.c:3099-3494; Gaussian :680-1289 or Matern-1/2 :2390-3033, as
 * set up last) over the data, windows and hyperparameters (_params[0] = f, _params[1] = l, _noise_level
 * = mu) of the additive handle `str`, landmarks perm[0..k-1] of the permutation perm[0..n-1]:
 * K11 + sqrt(k) ulp(|K11|_F) I = L L^T (chol.c:446-466), U1 = K(perm, perm[:k]) L^{-T},
 * U1^T U1 = V diag(w) V^T, U = U1 V w^{-1/2} (descending w), s = max(1/(w + eta), 0), eta = mu f^2.
 * The n x k panel and the n x k x k products run on the GPU (v_mfma_f64_16x16x4), the k x k Cholesky,
 * inverse and eigensolve on the GPU through rocSOLVER (dlopen'ed; host fallback when it is absent).  Returns a handle for Nfft4GPAmdNysSolve / Nfft4GPAmdNysFree, or
 * NULL (message on stderr) if K11 is not positive definite or the handle is unsuitable.
 * k11_mode 0 reproduces the reference's K11 exactly: nys.c:569 passes the k x d sub-data to the additive
 * kernel, which ignores it and reads its own gathered buffer at window stride k*dwindows (kernels.c:3160),
 * so K11 is built from buffer slices, not from the landmarks.  k11_mode 1 uses K(perm[:k], perm[:k]). */
void *Nfft4GPAmdNysSetupAdditive(void *str, const int *perm, int k, int k11_mode);
/* copy a Nystrom handle's factors to the host: U (n x k column-major) with rows in the order of perm
 * (pass the setup's perm to get the reference's permuted row order, NULL for natural order), s (k),
 * eta; any output may be NULL */
int Nfft4GPAmdNysFactors(void *nys, const int *perm, NFFT4GP_DOUBLE *U, NFFT4GP_DOUBLE *s, NFFT4GP_DOUBLE *eta);
/* storage of U read by Nfft4GPAmdNysSolve: 64 (default, the reference's fp64) or 32 (an fp32 copy, half the
 * bytes of the two HBM-bound passes; accumulation stays fp64).  The preconditioner only steers PCG, whose
 * stopping test is on the true fp64 residual (pcg.c:181-193), so fp32 storage changes the iteration
 * count at most, not the accuracy of the solution.  Returns 0 or -1. */
int Nfft4GPAmdNysSetStorage(void *nys, int bits);
/* hipEvent durations (ms) of a GPU setup's four big kernels: the panel, U1 = Kp G^T, the Gram U1^T U1 and
 * U = U1 W (the three MFMA products, 2 n k^2 flops each); zeros for a handle from Nfft4GPAmdNysCreate */
int Nfft4GPAmdNysSetupTimes(void *nys, NFFT4GP_DOUBLE *ms4);

/* ---- Nystrom preconditioner with gradients, the reference's interface (SRC/preconds/nys.h:62-179) -----
 * Drop-ins for Nfft4GPPrecondNysCreate / Free / Reset / SetRank / SetPerm (nys.c:3-113),
 * Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660, a precond_kernel_setup), Nfft4GPPrecondNysSolve
 * (func_solve, nys.c:115-173), Nfft4GPPrecondNysDvp (func_dvp, nys.c:175-330), Nfft4GPPrecondNysTrace
 * (func_trace, nys.c:332-474) and Nfft4GPPrecondNysLogdet (func_logdet, nys.c:476-500), for
 * Nfft4GPGpLoss's precond_* arguments (gp_loss.c:96-307).  The setup's fkernel must be this library's
 * Nfft4GPNFFTAdditiveKernelGaussianKernel / ...Matern12Kernel and fkernel_params an additive handle of this
 * library (its gathered windows _buffer and _params / _noise_level play the role of the reference's dense
 * additive kernel data, kernels.c:3099-3494; the reference's own Nfft4GPKernelAdditiveKernel is not part of
 * this library).  Factors, panels and gradients stay in HBM; Solve / Dvp take host or device vectors
 * (Dvp allocates *yp like the reference when it is NULL, on the side x lives on).
 * Nfft4GPAmdPrecondNysSetK11Mode: 0 (default) = the reference's K11 (see Nfft4GPAmdNysSetupAdditive),
 * 1 = K(perm[:k], perm[:k]) with the gradient panels over every window. */
void *Nfft4GPAmdPrecondNysCreate(void);
void Nfft4GPAmdPrecondNysFree(void *str);
void Nfft4GPAmdPrecondNysReset(void *str);
void Nfft4GPAmdPrecondNysSetRank(void *str, int k);
void Nfft4GPAmdPrecondNysSetPerm(void *str, int *perm, int own_perm);
void Nfft4GPAmdPrecondNysSetK11Mode(void *str, int mode);
int Nfft4GPAmdPrecondNysSetupWithKernel(NFFT4GP_DOUBLE *data, int n, int ldim, int d, func_kernel fkernel,
                                        void *fkernel_params, int require_grad, void *vnys_mat);
int Nfft4GPAmdPrecondNysSolve(void *vnys_mat, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
int Nfft4GPAmdPrecondNysDvp(void *vnys_mat, int n, int *mask, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE **yp);
int Nfft4GPAmdPrecondNysTrace(void *vnys_mat, NFFT4GP_DOUBLE **tracesp);
NFFT4GP_DOUBLE Nfft4GPAmdPrecondNysLogdet(void *vnys_mat);

/* ---- the reference's own Nystrom struct and apply, under the reference's name --------------------------
 * precond_nys: field layout identical to SRC/preconds/nys.h:24-55 (INC/_preconds.h:320-351; offsets tested in
 * tests/test_dropin.py).  The Cholesky factor stays opaque (SRC/preconds/chol.h:18).
 * Nfft4GPPrecondNysSolve replaces the reference's (INC/_preconds.h:400, nys.c:115-173): x = M^{-1} rhs,
 * M^{-1} = U S U^T + (I - U U^T) / eta in the permuted order of _perm, a func_solve.  vnys_mat is either
 * a precond_nys built by the reference's own Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660; host _U, _s,
 * _perm, _eta, _n, _k are read at the offsets above), or a handle of Nfft4GPAmdPrecondNysCreate (then it is
 * Nfft4GPAmdPrecondNysSolve).  A reference struct's factors are mirrored into HBM on first use (U stored
 * un-permuted, as Nfft4GPAmdNysCreate does) and the mirror is reused while _U, _s, _perm, _n, _k, _eta,
 * _tset and a fingerprint of s and of sampled U and perm entries are unchanged (a re-setup rebuilds it);
 * at most two mirrors are kept (least recently used first out).  x and rhs may be host or device
 * arrays; n is ignored like the reference (it reads _n).  _titt / _tits are updated as nys.c:166-170 does.
 * The reference's setup, Dvp, Trace and Logdet keep their host implementation (they run on the dense
 * kernel callbacks of the caller and on its host-side _K / _dU / _chol_K11); the Dvp's own applies
 * (nys.c:289, :312) reach this Solve through the dynamic linker when this library is linked first. */
typedef struct NFFT4GP_PRECOND_CHOL_STRUCT *pprecond_chol;
typedef struct NFFT4GP_PRECOND_NYS_STRUCT
{
   int _k_setup;
   int _own_perm;
   int *_perm;
   int _n;
   int _tits;
   NFFT4GP_DOUBLE _titt;
   NFFT4GP_DOUBLE _tset;
   NFFT4GP_DOUBLE _tlogdet;
   NFFT4GP_DOUBLE _tdvp;
   int _nys_opt;
   int _k;
   NFFT4GP_DOUBLE _eta;
   NFFT4GP_DOUBLE _f2;
   NFFT4GP_DOUBLE *_U;
   NFFT4GP_DOUBLE *_s;
   NFFT4GP_DOUBLE *_work;
   NFFT4GP_DOUBLE *_K;
   NFFT4GP_DOUBLE *_dU;
   NFFT4GP_DOUBLE *_dK;
   pprecond_chol _chol_K11;
   int _dvp_nosolve;
} precond_nys, *pprecond_nys;
int Nfft4GPPrecondNysSolve(void *vnys_mat, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
/* drop the HBM mirror kept for a reference precond_nys (e.g. before the caller frees it); 0 if none */
int Nfft4GPAmdPrecondNysMirrorRelease(void *vnys_mat);

/* ---- FSAI preconditioner built on the GPU, with gradients (SRC/preconds/fsai.h:46-207) ----------------
 * Drop-ins for Nfft4GPPrecondFsaiCreate / Free / Reset / SetLfil (fsai.c:3-104),
 * Nfft4GPPrecondFsaiSetupWithKernel (fsai.c:302-673: KNN pattern kernels.c:121-278, per-row Cholesky
 * solves, gradients), Nfft4GPPrecondFsaiSolve (func_solve, :106-123), Nfft4GPPrecondFsaiDvp (func_dvp,
 * :125-216), Nfft4GPPrecondFsaiTrace (func_trace, :218-276), Nfft4GPPrecondFsaiLogdet (func_logdet,
 * :278-301) and the CSR triangular solves Nfft4GPPrecondFsaiInvL / InvLT (:675-728), level-scheduled on
 * the device.  The setup's kernel is the plain Gaussian (default, or fkernel ==
 * Nfft4GPNFFTAdditiveKernelGaussianKernel) or Matern-1/2 (Nfft4GPAmdPrecondFsaiSetKernel(.., 1), or fkernel
 * == Nfft4GPNFFTAdditiveKernelMatern12Kernel) kernel of all d columns of data, with _params[0] = f,
 * _params[1] = l, _noise_level = mu read from fkernel_params (any struct with the nfft4gp_kernel layout,
 * the reference's Nfft4GPKernelParamCreate handle included); lfil <= 64, d <= 256.
 * Nfft4GPAmdPrecondFsaiSetCsr loads given factors (e.g. the reference's _L_i, _L_j, _L_a, _dL_a; da may be
 * NULL); Nfft4GPAmdPrecondFsaiCsr copies them out (any output may be NULL) and returns nnz. */
void *Nfft4GPAmdPrecondFsaiCreate(void);
void Nfft4GPAmdPrecondFsaiFree(void *str);
void Nfft4GPAmdPrecondFsaiReset(void *str);
void Nfft4GPAmdPrecondFsaiSetLfil(void *str, int lfil);
void Nfft4GPAmdPrecondFsaiSetKernel(void *str, int kernel);
int Nfft4GPAmdPrecondFsaiSetupWithKernel(NFFT4GP_DOUBLE *data, int n, int ldim, int d, func_kernel fkernel,
                                         void *fkernel_params, int require_grad, void *vfsai_mat);
int Nfft4GPAmdPrecondFsaiSetCsr(void *vfsai_mat, int n, const int *ia, const int *ja, const NFFT4GP_DOUBLE *aa,
                                const NFFT4GP_DOUBLE *da);
int Nfft4GPAmdPrecondFsaiCsr(void *vfsai_mat, int *ia, int *ja, NFFT4GP_DOUBLE *aa, NFFT4GP_DOUBLE *da);
int Nfft4GPAmdPrecondFsaiSolve(void *vfsai_mat, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
int Nfft4GPAmdPrecondFsaiInvL(void *vfsai_mat, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
int Nfft4GPAmdPrecondFsaiInvLT(void *vfsai_mat, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
int Nfft4GPAmdPrecondFsaiDvp(void *vfsai_mat, int n, int *mask, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE **yp);
int Nfft4GPAmdPrecondFsaiTrace(void *vfsai_mat, NFFT4GP_DOUBLE **tracesp);
NFFT4GP_DOUBLE Nfft4GPAmdPrecondFsaiLogdet(void *vfsai_mat);

/* ---- FSAI preconditioner apply (SRC/preconds/fsai.c:106-123) --------------------------------------
 * The reference's Nfft4GPPrecondFsaiSetupWithKernel (fsai.c:333-...) produces the lower-triangular
 * factor L in CSR (precond_fsai _L_i, _L_j, _L_a; fsai.h:11-58).  Nfft4GPAmdFsaiCreate takes those
 * three host arrays (n+1, nnz, nnz) and keeps L and L^T in HBM. */
void *Nfft4GPAmdFsaiCreate(int n, const int *L_i, const int *L_j, const NFFT4GP_DOUBLE *L_a);
/* same signature and result as Nfft4GPPrecondFsaiSolve (fsai.c:106): x = L^T (L rhs); each row is summed
 * in the reference's order with unfused multiply-adds, so x is bitwise the reference's */
int Nfft4GPAmdFsaiSolve(void *fsai, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
void Nfft4GPAmdFsaiFree(void *fsai);

/* ---- AFN preconditioner apply (SRC/preconds/afn.c:82-143) -----------------------------------------
 * precond_afn (afn.h:14-85) holds perm (n), the Cholesky factor of A11 = K(perm[:k], perm[:k]) + noise
 * (k x k lower, column-major), K12 = K(perm[:k], perm[k:]) (k x (n-k) column-major) and the FSAI of the
 * Schur complement (an Nfft4GPAmdFsaiCreate handle of size n-k, not owned).  0 <= k <= n: k = 0 applies
 * the FSAI alone, k = n solves with A11 on the unpermuted rhs, as afn.c:101-110 does.  AFN is not in the
 * reference's build (Makefile:3-26 lists chol, fsai, nys only); this is its apply. */
void *Nfft4GPAmdAfnCreate(int n, int k, const int *perm, const NFFT4GP_DOUBLE *L11, const NFFT4GP_DOUBLE *K12,
                          void *fsai_schur);
/* same signature as Nfft4GPPrecondAFNSolve (afn.c:82) */
int Nfft4GPAmdAfnSolve(void *afn, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
void Nfft4GPAmdAfnFree(void *afn);
/* AFN setup on the device: Nfft4GPPrecondAFNSetup (afn.c:161-489) with rank k given (its rank estimation,
 * afn.c:178-243 / rankest.c, is the caller's), schur_opt 3 (kernel FSAI of the Schur complement through
 * Nfft4GPKernelSchurCombineKernel, kernels.c:3496-3760; lfil = schur_lfil <= 64) and the ordering
 * perm_opt 0: identity (afn.c:245-256), 1: farthest points (Nfft4GPAmdSortFps, afn.c:196-209), 2: perm (n
 * entries, e.g. the reference's Nfft4GPRandPerm expanded, afn.c:210-218).  kernel: 0 Gaussian
 * (Nfft4GPKernelGaussianKernel), 1 Matern-1/2; fkernel_params: an nfft4gp_kernel (_params[0] = f,
 * _params[1] = l, _noise_level = mu).  data: host or device, n x d column-major (ldim).  Returns a handle
 * for Nfft4GPAmdAfnSolve / Nfft4GPAmdAfnFree (which then also frees the Schur FSAI), NULL on error. */
void *Nfft4GPAmdAfnSetup(const NFFT4GP_DOUBLE *data, int n, int ldim, int d, int k, int perm_opt, const int *perm,
                         int schur_lfil, int kernel, void *fkernel_params);
/* the same with the reference's schur_opt (afn.c:449-480): 3 as above, 0 the scaled identity
 * S^{-1} = I / _noise_level (afn.c:451-459, k > 0).  fkernel_params may also be this library's additive
 * NFFT handle (after its setup): the kernel is then the dense additive kernel of its window buffer and
 * hyperparameters (kernels.c:3099-3494, the points' K(perm[:k], .) -- not the reference's buffer-row
 * quirk), the FPS order and the KNN pattern still come from data. */
void *Nfft4GPAmdAfnSetupSchur(const NFFT4GP_DOUBLE *data, int n, int ldim, int d, int k, int perm_opt,
                              const int *perm, int schur_opt, int schur_lfil, int kernel, void *fkernel_params);
/* The AFN apply's two K12 products (K12^T y1 and K12 y2, afn.c:82-143) as matvecs of this library's additive
 * NFFT handle op (whole rows, set up over the AFN's n points with its kernel -- the handle the AFN was built
 * from): the landmark (Schur) part of the permuted vector placed at its points, zero elsewhere, through
 * Nfft4GPAdditiveNFFTMatSymv's operator and read back at the other part's points (the operator's mu term meets
 * only zeros there).  The products then carry the NFFT operator's approximation of the dense kernel
 *  instead of the stored K12's values, at two matvecs per apply instead of two passes over
 * k (n - k) doubles.  op NULL: back to the stored K12.  op must stay alive while the AFN applies.  An AFN
 * set up with gradients keeps the stored K12 (its Dvp / Trace / Logdet describe those factors).  0 / -1. */
int Nfft4GPAmdAfnSetOperator(void *afn, void *op);
/* the AFN handle's rank, permutation (n) and Schur-complement FSAI (CSR, n - k rows); any output may be
 * NULL; returns the FSAI's nnz (0 without one), -1 on error */
int Nfft4GPAmdAfnInfo(void *afn, int *k, int *perm, int *ia, int *ja, NFFT4GP_DOUBLE *aa);

/* ---- rank estimation (SRC/linearalg/rankest.c) -----------------------------------------------------
 * Drop-ins for Nfft4GPRankestNysScaled (rankest.c:248-391: nsample_r scaled subsamples of nsample points
 * drawn with libc rand() as Nfft4GPRandPerm does, FPS-ordered, the Nystrom error of ranks 0, ngap, ... on
 * each) and Nfft4GPRankestDefault (rankest.c:30-181: fill-distance / eigenvalue tolerance from
 * subsamples, then FPS of the full data up to max_rank; perm receives the selected points), with the
 * rankest struct's fields as arguments (reference defaults: max_rank 2000, nsample 500, nsample_r 5,
 * full_tol 0.9).  kernel 0 Gaussian, 1 Matern-1/2; fkernel_params an nfft4gp_kernel, or this library's
 * additive NFFT handle (the subsamples' kernel matrices are then its dense additive kernel).  The FPS passes,
 * kernel matrices, Cholesky / inverse / eigenvalues (rocSOLVER) and Nystrom products (MFMA GEMM) run on
 * the device; they consume rand() exactly as the reference does, so after the same srand() both pick the
 * same subsamples.  A rank-k factor of a subsample that is not positive definite counts as error
 * infinity (the reference continues on the partial factor).  Return the rank, -1 on error. */
int Nfft4GPAmdRankestNysScaled(const NFFT4GP_DOUBLE *data, int n, int ldim, int d, int kernel, void *fkernel_params,
                               int max_rank, int nsample, int nsample_r);
int Nfft4GPAmdRankestDefault(const NFFT4GP_DOUBLE *data, int n, int ldim, int d, int kernel, void *fkernel_params,
                             int max_rank, int nsample, int nsample_r, NFFT4GP_DOUBLE full_tol, int *perm);
/* The rank and ordering step of Nfft4GPPrecondAFNSetup (afn.c:165-256) with max_k, perm_opt (0 random,
 * 1 FPS) and nsamples as there: returns k and writes the full permutation (n entries, the k selected
 * points first).  k == max_k: pass k and perm to Nfft4GPAmdAfnSetup (perm_opt 2); 0 < k < max_k: the
 * reference builds a rank-k Nystrom instead (afn.c:287-296). */
int Nfft4GPAmdAfnRankEstimate(const NFFT4GP_DOUBLE *data, int n, int ldim, int d, int max_k, int perm_opt,
                              int nsamples, int kernel, void *fkernel_params, int *perm);
/* Nfft4GPPrecondAFNSetup (afn.c:161-489) in one call, its arguments as there (kernel: 0 Gaussian, 1
 * Matern-1/2; fkernel_params an nfft4gp_kernel or this library's additive NFFT handle):
 * Nfft4GPAmdAfnRankEstimate, then the AFN with that rank and order (k == max_k, k == 0, k == n), or
 * the rank-k Nystrom on the estimated landmarks when 0 < k < max_k (afn.c:294-304, MATLAB afn_setup.m:80-83),
 * or -- when the AFN's factors break down (K11 not positive definite, the Schur FSAI meets a non-positive
 * pivot) -- MATLAB's RAN fallback, a Nystrom on the same order (afn_setup.m:93-98).  Nfft4GPAmdPrecondAFNSolve
 * is the func_solve of whichever was built; Nfft4GPAmdPrecondAFNInfo reports kind (0 AFN, 1 Nystrom below
 * max_k, 2 Nystrom after a breakdown; with gradients 3 FSAI at k = 0, 4 Nystrom at k = n), k and the
 * underlying Nfft4GPAmdAfn* / Nfft4GPAmdNys* handle. */
void *Nfft4GPAmdPrecondAFNSetup(const NFFT4GP_DOUBLE *data, int n, int ldim, int d, int max_k, int perm_opt,
                                int schur_opt, int schur_lfil, int nsamples, int kernel, void *fkernel_params,
                                int require_grad);
int Nfft4GPAmdPrecondAFNSolve(void *pre, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
int Nfft4GPAmdPrecondAFNInfo(void *pre, int *kind, int *k, void **afn, void **nys);
void Nfft4GPAmdPrecondAFNFree(void *pre);
/* The same preconditioner behind the interface Nfft4GPGpLoss takes (gp_loss.c:96-307: precond_kernel_setup,
 * func_solve, func_trace, func_logdet, func_dvp, reset): Create keeps the parameters, SetupWithKernel
 * rebuilds on every loss call (fkernel Nfft4GPNFFTAdditiveKernelMatern12Kernel selects Matern-1/2, anything
 * else the Gaussian).  With require_grad the AFN keeps its gradient pieces -- MATLAB afn_setup.m / afn_dvp.m /
 * afn_trace.m / afn_logdet.m; the reference's C afn.c has none: dL11 = L Phi(L^{-1} dK11 L^{-T}), dK12, the
 * Schur FSAI's dG from the Schur kernel's gradient (schurCombinedKernelMat.m) -- and the Nystrom branches
 * are Nfft4GPAmdPrecondNys* with gradients (additive handle as kernel data).  Dvp returns
 * M^{-1} (dM/dtheta_g) x like the reference's nys.c / fsai.c (afn_dvp.m returns (dM/dtheta_g) x: the
 * result goes through the apply once more); Trace = tr(M^{-1} dM/dtheta_g), Logdet = log det M.
 * AFN gradients need schur_opt 3.  With gradients the k = n and k = 0 branches (afn.c:263-284) are built as
 * their exact equivalents that have gradients: kind 4, the rank-n Nystrom (= K + mu f^2 I), and kind 3, the
 * FSAI of the whole kernel (Nfft4GPAmdPrecondFsai*, lfil schur_lfil); Info reports them. */
void *Nfft4GPAmdPrecondAFNCreate(int max_k, int perm_opt, int schur_opt, int schur_lfil, int nsamples);
int Nfft4GPAmdPrecondAFNSetupWithKernel(NFFT4GP_DOUBLE *data, int n, int ldim, int d, func_kernel fkernel,
                                        void *fkernel_params, int require_grad, void *pre);
int Nfft4GPAmdPrecondAFNDvp(void *pre, int n, int *mask, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE **yp);
int Nfft4GPAmdPrecondAFNTrace(void *pre, NFFT4GP_DOUBLE **tracesp);
NFFT4GP_DOUBLE Nfft4GPAmdPrecondAFNLogdet(void *pre);
void Nfft4GPAmdPrecondAFNReset(void *pre);

/* ---- farthest point sampling (SRC/linearalg/ordering.c) -------------------------------------------
 * Nfft4GPSortFps with kFpsAlgorithmParallel1 (ordering.c:422-739): *k in: the number of points to select
 * (<= 0: all n), out: the number selected (fewer when the fill distance falls below tol); perm and dist
 * (may be NULL): host arrays of *k entries receiving the selected points and their fill distances
 * (the reference's _dist).  data: host or device, n x d column-major (ldim), d <= 256. */
int Nfft4GPAmdSortFps(const NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *k, NFFT4GP_DOUBLE tol, int *perm,
                      NFFT4GP_DOUBLE *dist);

/* ---- MI355X extensions --------------------------------------------------------------------------- */
/* stream every kernel of this library is enqueued on (hipStream_t; NULL = null stream) */
void Nfft4GPAmdSetStream(void *hip_stream);
void *Nfft4GPAmdGetStream(void);
/* 1 if a HIP device is visible */
int Nfft4GPAmdDeviceAvailable(void);
/* library version string */
const char *Nfft4GPAmdVersion(void);

/* layout statistics of an additive handle after its first setup:
 * out[0]=n, [1]=nwindows, [2]=block size, [3]=#blocks, [4]=#tiles, [5]=slots (incl. padding),
 * [6]=points per chunk R, [7]=comps per group, [8]=#groups, [9]=device bytes of the layout */
int Nfft4GPAmdAdditiveLayoutInfo(void *str, long long *out, int nout);

/* per-kernel timing with hipEvents on the library stream (0 disables; resets counters when enabled).
 * After enabling, every additive matvec launches its spread / grid / interp kernels with start / stop
 * events attached to the dispatches (hipExtLaunchKernelGGL: the dispatch packet's own begin / end
 * timestamps, the durations rocprofv3's kernel trace reports; multi-feature windows: events recorded
 * around each launch).
 * Nfft4GPAmdTimingQuery writes total milliseconds and launch counts for the three kernels:
 * ms[0..2] = spread, grid, interp;  cnt[0..2] likewise.  Returns 0. */
int Nfft4GPAmdTimingEnable(void *str, int enable);
/* deterministic 1-D matvec (off by default; env NFFT4GP_AMD_DET=1): the spread's moment-table flushes and the
 * interpolation's y adds are rounded, before their LDS atomics, to a grid on which every partial sum is exact, so
 * the result does not depend on the order the waves add in -- two matvecs of one vector are bitwise equal, and so
 * are two PCG runs.  Costs ~2^-45 relative rounding of each cell's moments and y value, and ~11 % of the matvec
 * at config C.  0: plain fp64 LDS atomics, reproducible to rounding. */
int Nfft4GPAmdSetDeterministic(void *str, int on);
/* 32-bit precision mode of a 1-D additive handle (bits 32; 64 = the default), the analogue of the reference's
 * NFFT4GP_USING_FLOAT32 (SRC/utils/utils.h:28-31) for BASELINE configs[4]: each (point, window) is ONE 32-bit
 * record -- the offset in the cell to 2^-21 of a cell (2^-27 of the period, finer than an fp32 coordinate) with the
 * 12-bit local index in its low bits -- instead of 5 bytes, a fifth fewer bytes per pass; the arithmetic stays fp64.
 * Matches the reference to ~1e-7 (tests/test_gpu_precision.py; the fp64 default to ~1e-9).  The layout is rebuilt
 * (and the kernel re-set up) when called after the first setup; env NFFT4GP_AMD_PRECISION=32.  Multi-feature
 * windows are unaffected. */
int Nfft4GPAmdSetPrecision(void *str, int bits);
int Nfft4GPAmdTimingQuery(void *str, double *ms, long long *cnt);
/* average duration of ONE kernel of the additive matvec (which: 0 spread, 1 grid, 2 interp), measured
 * with a single hipEvent pair around `reps` back-to-back launches on the library stream (per-launch
 * event pairs add several microseconds each).  x, y: device vectors of the handle's size (y: 3n if
 * grad).  Writes the mean milliseconds per launch. */
int Nfft4GPAmdKernelBench(void *str, int which, int grad, int reps, const NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *y,
                          double *ms_avg);

/* split-phase additive matvec for row-sharded multi-GPU use (one process per GPU):
 *   phase 1 (spread): per-component oversampled-grid partial sums of this rank's points into grid
 *                     (device, Nfft4GPAmdShardGridSize doubles, overwritten);
 *   -- caller all-reduces grid across ranks (RCCL) --
 *   phase 2 (finish): circulant + interpolation + epilogue for this rank's points.
 * The handle must have been created with Nfft4GPAmdAdditiveShardCreate.  x, y are device pointers to
 * this rank's rows.  grad = 0: y has n_local entries; grad = 1: y has 3*n_local (y0|y1|y2). */
void *Nfft4GPAmdAdditiveShardCreate(NFFT4GP_DOUBLE *data, int n_global, int ldim, int d, int *windows,
                                    int nwindows, int dwindows, int row_begin, int row_end);
int Nfft4GPAmdShardSpread(void *str, const NFFT4GP_DOUBLE *x_local, NFFT4GP_DOUBLE *grid);
int Nfft4GPAmdShardFinish(void *str, const NFFT4GP_DOUBLE *grid, int grad, NFFT4GP_DOUBLE alpha,
                          const NFFT4GP_DOUBLE *x_local, NFFT4GP_DOUBLE beta, NFFT4GP_DOUBLE *y_local);
/* elements of the grid Nfft4GPAmdShardSpread writes and Nfft4GPAmdShardFinish reads: nwindows * 64 when
 * every window is 1-D, nwindows * 64^dmax otherwise (the real spread grids of multi-feature windows) */
long long Nfft4GPAmdShardGridSize(void *str);

/* ---- multi-GPU operators (one process per GPU) ----------------------------------------
 * The reference is single-process: its additive matvec loops the components sequentially into _dwork
 * (nfft_interface.c:796-817) and its PCG (pcg.c:3-206) works on whole vectors.  Here the operator is
 * split over a communicator and stays a func_symmatvec, so Nfft4GPSolverPcg drives it unchanged.
 *
 * Communicators.  Nfft4GPAmdCommCreateRccl: RCCL over xGMI (librccl, the copy PyTorch mapped), every
 * all-reduce enqueued on the library stream; rank 0 makes the id with Nfft4GPAmdCommUniqueId (128 bytes)
 * and the caller broadcasts it.  Nfft4GPAmdCommCreateCallback: the caller's all-reduce (e.g. a gloo
 * process group), called with a device staging buffer of `capacity` doubles it owns; it must leave the
 * elementwise sum over the ranks in place.  Both return NULL on failure. */
typedef int (*Nfft4GPAmdAllreduceFn)(void *ctx, NFFT4GP_DOUBLE *d_buf, long long count);
int Nfft4GPAmdCommRcclAvailable(void);  /* 1: this process can create an RCCL communicator */
int Nfft4GPAmdCommUniqueId(void *id128);
void *Nfft4GPAmdCommCreateRccl(int rank, int world, const void *id128);
void *Nfft4GPAmdCommCreateCallback(int rank, int world, Nfft4GPAmdAllreduceFn fn, void *ctx,
                                   NFFT4GP_DOUBLE *d_stage, long long capacity);
/* sum of count doubles at d_buf (device) over the ranks, in place, on the library stream */
int Nfft4GPAmdCommAllreduce(void *comm, NFFT4GP_DOUBLE *d_buf, long long count);
void Nfft4GPAmdCommFree(void *comm);
/* ranks the communicator's backend itself reports: ncclCommCount for RCCL, the group size for a callback */
int Nfft4GPAmdCommRanks(void *comm);

/* Component shard: a whole-row additive handle over a subset of the windows, weighted 1/nw_global (the
 * whole operator's 1/nwindows, nfft_interface.c:806); own_diag = 1 on exactly one rank, which adds the
 * mu x term (and the gradient's f^2 x block).  Call before the kernel setup.  The ranks' y sum to the
 * whole operator's. */
int Nfft4GPAmdAdditiveComponentShard(void *str, int nw_global, int own_diag);
/* Distributed operator over `comm`.  kind 0 (rows): `handle` from Nfft4GPAmdAdditiveShardCreate; x, y
 * hold this rank's rows; one all-reduce of the Nfft4GPAmdShardGridSize grid per matvec.  kind 1
 * (components): `handle` a component shard; x, y are whole (replicated) vectors; one all-reduce of y
 * (n, 3n for the gradient) per matvec.  Free it before its handle and communicator. */
void *Nfft4GPAmdDistCreate(void *handle, int kind, void *comm);
void Nfft4GPAmdDistFree(void *dop);
/* func_symmatvec on device vectors (n = this rank's rows for kind 0, n_global for kind 1).  Given to
 * Nfft4GPSolverPcg, the solver sums its dot products over the communicator (kind 0) and clamps maxits
 * to the global n, so its iterations equal the single-GPU solver's up to rounding. */
int Nfft4GPAmdDistMatSymv(void *dop, int n, NFFT4GP_DOUBLE alpha, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE beta,
                          NFFT4GP_DOUBLE *y);
/* synchronise the library stream, then 0, or -1 (message on stderr) if a peer exchange of this operator timed
 * out in the work enqueued so far: its y are then not to be used.  The solvers (PCG, FGMRES, Lanczos, the
 * quadrature, the loss) make this check before they report success. */
int Nfft4GPAmdDistCheck(void *dop);
/* kind 1 (components): y is all-reduced in `chunks` pieces (default 4) on a stream of the operator's own,
 * each piece as soon as the interpolation launch that writes it is done, so the all-reduce of piece i
 * overlaps the interpolation of piece i + 1 (1-D windows, plain matvec; the gradient matvec and
 * multi-feature windows all-reduce y once).  chunks = 1: one all-reduce after the matvec.  The sums are
 * the same element for element. */
int Nfft4GPAmdDistSetChunks(void *dop, int chunks);
/* kind 0 (rows), 1-D windows: replace the all-reduce of the grids by a peer-memory exchange (collective; call
 * on every rank after the kernel setup).  Each rank exports one device buffer (hipIpcGetMemHandle: two slots
 * of the nw x 64 grids and an arrival flag per window) and opens the others'; a matvec then writes its grids
 * into its own slot and publishes the flags (k_reduce_parts), and the grid kernel waits for every rank's
 * flags and sums the slots in rank order -- every rank holds the same bits, and there is no separate
 * all-reduce launch.  A wait gives up after NFFT4GP_AMD_PEER_SPIN polls (default 2^20, ~2 s): the call after
 * it returns -1.  Returns 0 (on), 1 (not applicable: kind 1 or multi-feature windows, on every rank alike)
 * or -1 (some rank could not allocate, export or open a buffer: every rank keeps the all-reduce).  With the
 * exchange on, Nfft4GPAmdDistFree is collective.  Replaces the grid all-reduce of the reference's sequential
 * component sum (nfft_interface.c:796-817) split over row shards; no reference counterpart. */
int Nfft4GPAmdDistPeerEnable(void *dop);
/* back to the communicator's all-reduce (collective; also after a wait gave up) */
int Nfft4GPAmdDistPeerDisable(void *dop);
/* 1 if the peer exchange is on, 0 if not, -1 for a NULL operator */
int Nfft4GPAmdDistPeerActive(void *dop);
/* per-rank timing of a distributed operator (0 disables; enabling resets): every matvec records hipEvents
 * on the library stream around this rank's kernels before the exchange, the all-reduce and the kernels
 * after it (kind 1: the local matvec, and each chunk's all-reduce on the operator's comm stream).
 * Query: ms[0..2] = total milliseconds of the three, *cnt = matvecs timed. */
int Nfft4GPAmdDistTimingEnable(void *dop, int enable);
int Nfft4GPAmdDistTimingQuery(void *dop, double *ms, long long *cnt);
int Nfft4GPAmdDistGradMatSymv(void *dop, int n, NFFT4GP_DOUBLE alpha, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE beta,
                              NFFT4GP_DOUBLE *y);
/* func_kernel (kernels.h:49) of a distributed operator, for Nfft4GPGpLoss (gp_loss.c:96-307): dop begins
 * with an nfft4gp_kernel header, so the loss writes _params[0] (f), _params[1] (l) and _noise_level (mu)
 * into it as it does into the reference's handle (gp_loss.c:143-150); the setup hands them to the local
 * handle (Nfft4GPNFFTAdditiveKernelGaussianKernel / ...Matern12Kernel, nfft_interface.c:676-794) and
 * returns *Kp = *dKp = dop.  With matvec = Nfft4GPAmdDistMatSymv and dmatvec = Nfft4GPAmdDistGradMatSymv
 * the loss, Nfft4GPSolverFgmres and Nfft4GPSolverLanczos run on the split operator: for kind 0 (rows)
 * n, label and the Rademacher probes are this rank's rows (probes column-major with stride n) and every
 * dot product and norm is summed over the communicator; kind 1 (components) has whole vectors. */
int Nfft4GPAmdDistGaussianKernel(void *dop, NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *permr, int kr,
                                 int *permc, int kc, NFFT4GP_DOUBLE **Kp, NFFT4GP_DOUBLE **dKp);
int Nfft4GPAmdDistMatern12Kernel(void *dop, NFFT4GP_DOUBLE *data, int n, int ldim, int d, int *permr, int kr,
                                 int *permc, int kc, NFFT4GP_DOUBLE **Kp, NFFT4GP_DOUBLE **dKp);
/* Row-sharded Nystrom apply (nys.c:115-173 over row shards): keeps rows [row_begin, row_end) of a
 * Nystrom preconditioner's U (Nfft4GPAmdNysCreate / Nfft4GPAmdNysSetupAdditive; copied, the source may
 * be freed); the apply is a local U^T r, a k-vector all-reduce and a local U w + r/eta.  func_solve on
 * this rank's rows (device). */
void *Nfft4GPAmdNysShard(void *nys, int row_begin, int row_end, void *comm);
/* The Nystrom setup (Nfft4GPPrecondNysSetupWithKernel, nys.c:518-660, as Nfft4GPAmdNysSetupAdditive with
 * k11_mode 0 / 1) split over the row shards of a distributed operator (kind 0, after its kernel setup):
 * each rank forms the panel K(rows, perm[:k]) of its own rows, U1 = Kp L^{-T} and its partial Gram
 * U1^T U1 on MFMA; one k x k all-reduce sums the Gram (matops.c:65-137), rank 0's k x k factors are
 * broadcast, and each rank keeps U for its rows only (n/N x k).  perm: the global landmark order (the
 * first k entries are read), the same on every rank.  Returns a handle for Nfft4GPAmdDistNysSolve /
 * Nfft4GPAmdDistNysFree. */
void *Nfft4GPAmdNysShardSetupAdditive(void *dop, const int *perm, int k, int k11_mode);
int Nfft4GPAmdDistNysSolve(void *dnys, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
void Nfft4GPAmdDistNysFree(void *dnys);
/* Row-sharded AFN apply (afn.c:82-143 over row shards): from an AFN apply handle (Nfft4GPAmdAfnCreate /
 * Nfft4GPAmdAfnSetup*, or the AFN of Nfft4GPAmdPrecondAFNInfo; 0 < k < n), this rank keeps the points of
 * rows [row_begin, row_end): its landmarks, the K12 columns of its Schur-complement points (k x ~(n-k)/N)
 * and their rows of the Schur FSAI G and of G^T.  An apply exchanges the rhs's landmark entries and the
 * K12 y2 partial sums (two k all-reduces) and, with the Schur FSAI, the Schur vector before each sparse
 * product (two (n-k) all-reduces of zero-padded vectors).  func_solve on this rank's rows (device). */
/* The AFN apply's two K12 passes (2 x 8 k (n - k) bytes, most of an apply) read an fp32 copy of K12 with
 * fp64 accumulation (bits 32), or the fp64 K12 (64, the default) -- Nfft4GPAmdNysSetStorage's analogue;
 * the preconditioner stays a fixed symmetric operator either way. */
int Nfft4GPAmdAfnSetStorage(void *afn, int bits);
/* The same choice for the setup flow's preconditioner: the AFN's K12 or the Nystrom branch's U (the
 * gradient-capable branches keep fp64). */
int Nfft4GPAmdPrecondAFNSetStorage(void *pre, int bits);
void *Nfft4GPAmdAfnShard(void *afn, int row_begin, int row_end, void *comm);
/* The same row shard set up on its own rank, with no full AFN anywhere (afn.c:161-489 split by rows, every
 * rank collectively): the ordering (perm_opt 0 identity, 1 FPS, 2 perm given; afn.c:196-256) and the k x k
 * factor of A11 are replicated (rank 0's L11^{-1} broadcast); each rank forms only the K12 columns of its own
 * Schur points (k x m2, afn.c:430-443), the KNN pattern of its own rows of the Schur FSAI (kernels.c:121-278:
 * scans over the earlier points of those rows only) and their values (fsai.c:302-670), with
 * W = L11^{-1} K12 formed chunk by chunk for the columns each chunk of rows touches.  G^T products sum each
 * rank's rows' contributions with one (n-k) all-reduce.  schur_opt 0 (S^-1 = I / mu) or 3 (kernel FSAI);
 * no gradients.  Apply / free with Nfft4GPAmdDistAfnSolve / Nfft4GPAmdDistAfnFree. */
void *Nfft4GPAmdAfnShardSetup(const NFFT4GP_DOUBLE *data, int n, int ldim, int d, int k, int perm_opt,
                              const int *perm, int schur_opt, int schur_lfil, int kernel, void *fkernel_params,
                              int row_begin, int row_end, void *comm);
/* what a row shard holds: its landmarks m1, its Schur points m2, K12 doubles (k m2), G entries */
int Nfft4GPAmdAfnShardInfo(void *dafn, int *m1, int *m2, long long *k12_doubles, long long *g_nnz);
int Nfft4GPAmdDistAfnSolve(void *dafn, int n, NFFT4GP_DOUBLE *x, NFFT4GP_DOUBLE *rhs);
void Nfft4GPAmdDistAfnFree(void *dafn);

/* ---- host-only helpers (no GPU needed): the setup math of the device plan, exported so the CPU
 * test-suite can check it and emulate the kernels against the oracle ------------------------------- */
/* tap polynomial coefficients C[t*NC + d], t = 0..9, d = 0..NC-1 (monomials in u = frac - 1/2);
 * returns NC, the coefficients per tap (C == NULL: only returns NC) */
int Nfft4GPAmdHostTapPoly(NFFT4GP_DOUBLE *C);
/* kernel kind 0 gaussian, 1 xx_gaussian, 2 laplacian_rbf, 3 der_laplacian_rbf with parameter c:
 * bhat[32] (k = -16..15) and the 64-point real circulant w = weight * sum_k bhat_k/phihut_k^2 cos(...) */
int Nfft4GPAmdHostCirculant(int kind, NFFT4GP_DOUBLE c, NFFT4GP_DOUBLE weight, NFFT4GP_DOUBLE *bhat,
                            NFFT4GP_DOUBLE *w);
/* centre + scale one 1-D window exactly as nfft_interface.c:150-213 and quantize to 32-bit fixed point;
 * returns the scale (or -1 if all points coincide) */
NFFT4GP_DOUBLE Nfft4GPAmdHostPrepare(const NFFT4GP_DOUBLE *col, int n, unsigned int *q);
/* chunk layout of per-window quantized coordinates qc[c*n + j] (B <= 4064); call with NULL arrays to
 * get counts[0] = ntiles, counts[1] = ngroups, counts[2] = nblocks, then with arrays of
 * ntiles*64 (meta), ntiles*4*64 (lo: local index bits 0-5, a byte per point), ntiles*16*64 (q: offset
 * in the cell in bits 0-25, local index bits 6-11 in bits 26-31), nblocks*ngroups+1 (tile_off) */
int Nfft4GPAmdHostLayout(const unsigned int *qc, int n, int nw, int B, int CG, long long *counts,
                         unsigned short *meta, unsigned int *lo, unsigned int *q, int *tile_off);
/* the same for either record (rec 5: the default, as above; rec 4: Nfft4GPAmdSetPrecision 32 -- no lo array,
 * q = the in-cell offset with the 12-bit local index in its low bits) */
int Nfft4GPAmdHostLayoutRec(const unsigned int *qc, int n, int nw, int B, int CG, int rec, long long *counts,
                            unsigned short *meta, unsigned int *lo, unsigned int *q, int *tile_off);
/* The same layout built on the GPU (layout_gpu.hip, what the operator's setup uses): identical arrays. */
int Nfft4GPAmdDeviceLayout(const unsigned int *qc, int n, int nw, int B, int CG, long long *counts,
                           unsigned short *meta, unsigned int *lo, unsigned int *q, int *tile_off);
int Nfft4GPAmdDeviceLayoutRec(const unsigned int *qc, int n, int nw, int B, int CG, int rec, long long *counts,
                              unsigned short *meta, unsigned int *lo, unsigned int *q, int *tile_off);
/* the Nystrom setup's host k x k steps: symmetric eigensolve (dsyev 'V' semantics: ascending w,
 * eigenvectors as the columns of V, column-major) and L^{-1} of the lower Cholesky factor of A + shift I
 * (returns 0, or the failing column + 1 if A + shift I is not positive definite) */
int Nfft4GPAmdHostSymEig(const NFFT4GP_DOUBLE *A, int n, NFFT4GP_DOUBLE *w, NFFT4GP_DOUBLE *V);
int Nfft4GPAmdHostCholInverse(const NFFT4GP_DOUBLE *A, int k, NFFT4GP_DOUBLE shift, NFFT4GP_DOUBLE *G);

#ifdef __cplusplus
}
#endif

#endif /* NFFT4GP_AMD_H */
