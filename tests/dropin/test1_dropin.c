/* test1_dropin.c -- TESTS/TEST1/foo.cpp:214-293 replayed as a C caller of the drop-in library.
 *
 * Compiled against include/nfft4gp_amd.h and linked  -lnfft4gp_amd  BEFORE the reference's own library
 * (oracle/_ref/libnfft4gp_ref.so, its dense path built from SRC/), the link order INTEGRATION.md gives:
 * the NFFT operator, the vector ops and the PCG resolve to libnfft4gp_amd, the dense additive kernel and
 * its SYMV to the reference.  Like foo.cpp it writes f, l, mu straight into the handles' fields, calls the
 * func_kernel setups with Kp / dKp, then compares the NFFT matvec and gradient matvec with the dense ones
 * on host vectors; it then solves with Nfft4GPSolverPcg on both operators.
 *
 * usage: test1_dropin n nwindows dwindows kernel(0 gauss, 1 matern) l mu tol_matvec
 * exit 0 when every check passes; the errors are printed in foo.cpp's format. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "nfft4gp_amd.h"

/* the reference's dense path (oracle/_ref), prototypes as in SRC/linearalg/kernels.h:275-290, :406-445 and
 * SRC/linearalg/matops.h:25-52 (the reference headers are not needed by the caller of this library) */
int Nfft4GPKernelGaussianKernel(void *str, double *data, int n, int ldim, int d, int *permr, int kr, int *permc,
                                int kc, double **Kp, double **dKp);
int Nfft4GPKernelMatern12Kernel(void *str, double *data, int n, int ldim, int d, int *permr, int kr, int *permc,
                                int kc, double **Kp, double **dKp);
void *Nfft4GPKernelAdditiveKernelParamCreate(double *data, int n, int ldim, int d, int *windows, int nwindows,
                                             int dwindows, func_kernel fkernel);
int Nfft4GPKernelAdditiveKernel(void *str, double *data, int n, int ldim, int d, int *permr, int kr, int *permc,
                                int kc, double **Kp, double **dKp);
int Nfft4GPDenseMatSymv(void *data, int n, double alpha, double *x, double beta, double *y);
int Nfft4GPDenseGradMatSymv(void *data, int n, double alpha, double *x, double beta, double *y);

static double rel_l2(const double *a, const double *b, int n)
{
   double e = 0.0, nb = 0.0;
   for (int i = 0; i < n; i++) {
      e += (a[i] - b[i]) * (a[i] - b[i]);
      nb += b[i] * b[i];
   }
   return sqrt(e) / sqrt(nb);
}

int main(int argc, char **argv)
{
   if (argc < 8) {
      fprintf(stderr, "usage: %s n nwindows dwindows kernel l mu tol\n", argv[0]);
      return 2;
   }
   const int n = atoi(argv[1]), nwindows = atoi(argv[2]), dwindows = atoi(argv[3]), kernel = atoi(argv[4]);
   const double l = atof(argv[5]), mu = atof(argv[6]), tol = atof(argv[7]);
   const int d = nwindows * dwindows;
   srand(906);
   double *X = (double *)malloc(sizeof(double) * (size_t)n * d);
   for (size_t i = 0; i < (size_t)n * d; i++) X[i] = (double)rand() / (double)RAND_MAX;
   int *windows = (int *)malloc(sizeof(int) * d);
   for (int i = 0; i < d; i++) windows[i] = i;

   /* foo.cpp:211-227 */
   func_kernel additivekernel = &Nfft4GPKernelAdditiveKernel;
   pnfft4gp_kernel additivekernel_data = (pnfft4gp_kernel)Nfft4GPKernelAdditiveKernelParamCreate(
       X, n, n, d, windows, nwindows, dwindows, kernel == 0 ? &Nfft4GPKernelGaussianKernel : &Nfft4GPKernelMatern12Kernel);
   func_kernel nfft_additivekernel =
       kernel == 0 ? &Nfft4GPNFFTAdditiveKernelGaussianKernel : &Nfft4GPNFFTAdditiveKernelMatern12Kernel;
   pnfft4gp_kernel nfft_additivekernel_data =
       (pnfft4gp_kernel)Nfft4GPNFFTAdditiveKernelParamCreate(X, n, n, d, windows, nwindows, dwindows);
   additivekernel_data->_params[0] = 1.0;
   additivekernel_data->_params[1] = l;
   additivekernel_data->_noise_level = mu;
   nfft_additivekernel_data->_params[0] = 1.0;
   nfft_additivekernel_data->_params[1] = l;
   nfft_additivekernel_data->_noise_level = mu;

   double *additive_mat = NULL, *additive_mat_grad = NULL;
   void *nfft_additive_mat = NULL, *nfft_additive_mat_grad = NULL;
   if (additivekernel((void *)additivekernel_data, X, n, n, d, NULL, 0, NULL, 0, &additive_mat, &additive_mat_grad) ||
       nfft_additivekernel((void *)nfft_additivekernel_data, X, n, n, d, NULL, 0, NULL, 0, (double **)&nfft_additive_mat,
                           (double **)&nfft_additive_mat_grad)) {
      fprintf(stderr, "kernel setup failed\n");
      return 1;
   }
   if (nfft_additive_mat != (void *)nfft_additivekernel_data || nfft_additive_mat_grad != nfft_additive_mat) {
      fprintf(stderr, "func_kernel must return the handle itself as Kp and dKp (nfft_interface.c:730-731)\n");
      return 1;
   }

   /* foo.cpp:229-254 */
   double *x_vec = (double *)malloc(sizeof(double) * n);
   double *y_nfft = (double *)calloc(n, sizeof(double)), *dy_nfft = (double *)calloc(3 * (size_t)n, sizeof(double));
   double *y_exact = (double *)calloc(n, sizeof(double)), *dy_exact = (double *)calloc(3 * (size_t)n, sizeof(double));
   /* re-seeded here: the HIP runtime's threads may draw libc rand() while the GPU initialises, so the
      sequence after the setups is not the seed's; the x drawn from a fresh seed is the same on every run */
   srand(907);
   Nfft4GPVecRand(x_vec, n);
   for (int i = 0; i < n; i++) x_vec[i] -= 0.5;
   if (Nfft4GPAdditiveNFFTMatSymv(nfft_additive_mat, n, 1.0, x_vec, 0.0, y_nfft) ||
       Nfft4GPAdditiveNFFTGradMatSymv(nfft_additive_mat_grad, n, 1.0, x_vec, 0.0, dy_nfft)) {
      fprintf(stderr, "NFFT matvec failed\n");
      return 1;
   }
   Nfft4GPDenseMatSymv(additive_mat, n, 1.0, x_vec, 0.0, y_exact);
   Nfft4GPDenseGradMatSymv(additive_mat_grad, n, 1.0, x_vec, 0.0, dy_exact);

   /* foo.cpp:256-293 (the L2 lines) */
   const double err = rel_l2(y_nfft, y_exact, n);
   double gerr[3];
   for (int j = 0; j < 3; j++) gerr[j] = rel_l2(dy_nfft + (size_t)j * n, dy_exact + (size_t)j * n, n);
   const double nrm = Nfft4GPVecNorm2(y_exact, n);
   printf("L2 Error. Rel: %24.20e (norm %e)\n", err, nrm);
   for (int j = 0; j < 3; j++) printf("L2 Gradient Error %d. Rel: %24.20e\n", j + 1, gerr[j]);
   int fail = !(err <= tol) || !(gerr[0] <= tol) || !(gerr[1] <= tol) || !(gerr[2] <= 1e-14);

   /* Nfft4GPSolverPcg (pcg.c:3-206) on the NFFT operator and on the reference's dense operator, host vectors */
   double *b = (double *)malloc(sizeof(double) * n), *x1 = (double *)calloc(n, sizeof(double));
   double *x2 = (double *)calloc(n, sizeof(double));
   for (int i = 0; i < n; i++) b[i] = x_vec[i];
   double rel1 = 0.0, rel2 = 0.0, *hist1 = NULL, *hist2 = NULL;
   int it1 = 0, it2 = 0;
   if (Nfft4GPSolverPcg(nfft_additive_mat, n, &Nfft4GPAdditiveNFFTMatSymv, NULL, NULL, x1, b, 2 * n, 0, 1e-6, &rel1,
                        &hist1, &it1, -1) ||
       Nfft4GPSolverPcg(additive_mat, n, &Nfft4GPDenseMatSymv, NULL, NULL, x2, b, 2 * n, 0, 1e-6, &rel2, &hist2, &it2,
                        -1)) {
      fprintf(stderr, "PCG failed\n");
      return 1;
   }
   const double xerr = rel_l2(x1, x2, n);
   printf("PCG NFFT: %d iterations, rel res %e; dense: %d iterations, rel res %e; solution rel diff %e\n", it1, rel1,
          it2, rel2, xerr);
   fail |= !(it1 > 0 && it2 > 0 && rel1 <= 1e-6 && rel2 <= 1e-6);

   Nfft4GPAdditiveNFFTKernelFree(nfft_additivekernel_data);
   free(hist1);
   free(hist2);
   free(X);
   free(windows);
   free(x_vec);
   free(y_nfft);
   free(dy_nfft);
   free(y_exact);
   free(dy_exact);
   free(b);
   free(x1);
   free(x2);
   printf(fail ? "FAIL\n" : "PASS\n");
   return fail;
}
