/* nys_dropin.c -- a TEST2-style caller (TESTS/TEST2/foo2.cpp:252-292, SRC/optimizer/gp_loss.c:51-74) of the
 * Nystrom preconditioner under the reference's own names: precond_nys built by the reference's
 * Nfft4GPPrecondNysCreate / SetPerm / SetRank / SetupWithKernel on its dense additive Gaussian kernel, then
 * handed as &Nfft4GPPrecondNysSolve to Nfft4GPSolverPcg with the reference's dense operator.
 *
 * Linked -lnfft4gp_amd first, Nfft4GPPrecondNysSolve and Nfft4GPSolverPcg resolve to libnfft4gp_amd (the GPU
 * apply reads the reference's struct); linked the reference first, both are the reference's.  The setup and
 * the Dvp stay the reference's in both orders; in the amd-first order the Dvp's own applies (nys.c:289, :312)
 * reach libnfft4gp_amd's Solve through the dynamic linker.
 *
 * usage: nys_dropin dir n d k f l mu require_grad
 *   dir holds X.bin (n x d column-major fp64), b.bin (n), perm.bin (n int32), rhs.bin (n); writes out.bin:
 *   [apply(rhs) (n) | apply by the reference's own Solve, looked up in its library (n) | PCG x (n) |
 *    iters, rel_res, tits | dvp(rhs) (3n, require_grad only)]
 * and prints which library Nfft4GPPrecondNysSolve came from. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nfft4gp_amd.h"

/* the reference's dense path and Nystrom setup (oracle/_ref), prototypes as in SRC/linearalg/kernels.h,
 * SRC/linearalg/matops.h and SRC/preconds/nys.h:62-157 */
int Nfft4GPKernelGaussianKernel(void *str, double *data, int n, int ldim, int d, int *permr, int kr, int *permc,
                                int kc, double **Kp, double **dKp);
void *Nfft4GPKernelAdditiveKernelParamCreate(double *data, int n, int ldim, int d, int *windows, int nwindows,
                                             int dwindows, func_kernel fkernel);
int Nfft4GPKernelAdditiveKernel(void *str, double *data, int n, int ldim, int d, int *permr, int kr, int *permc,
                                int kc, double **Kp, double **dKp);
int Nfft4GPDenseMatSymv(void *data, int n, double alpha, double *x, double beta, double *y);
void *Nfft4GPPrecondNysCreate(void);
void Nfft4GPPrecondNysFree(void *str);
void Nfft4GPPrecondNysSetRank(void *str, int k);
void Nfft4GPPrecondNysSetPerm(void *str, int *perm, int own_perm);
int Nfft4GPPrecondNysSetupWithKernel(double *data, int n, int ldim, int d, func_kernel fkernel, void *fkernel_params,
                                     int require_grad, void *vnys_mat);
int Nfft4GPPrecondNysDvp(void *vnys_mat, int n, int *mask, double *x, double **yp);

static void *load(const char *dir, const char *name, size_t bytes)
{
   char path[4096];
   snprintf(path, sizeof path, "%s/%s", dir, name);
   FILE *f = fopen(path, "rb");
   if (!f) {
      perror(path);
      exit(2);
   }
   void *p = malloc(bytes);
   if (fread(p, 1, bytes, f) != bytes) {
      fprintf(stderr, "%s: short read\n", path);
      exit(2);
   }
   fclose(f);
   return p;
}

int main(int argc, char **argv)
{
   if (argc < 9) {
      fprintf(stderr, "usage: %s dir n d k f l mu require_grad\n", argv[0]);
      return 2;
   }
   const char *dir = argv[1];
   const int n = atoi(argv[2]), d = atoi(argv[3]), k = atoi(argv[4]), grad = atoi(argv[8]);
   const double f = atof(argv[5]), l = atof(argv[6]), mu = atof(argv[7]);
   double *X = load(dir, "X.bin", sizeof(double) * (size_t)n * d);
   double *b = load(dir, "b.bin", sizeof(double) * n);
   int *perm = load(dir, "perm.bin", sizeof(int) * n);
   double *rhs = load(dir, "rhs.bin", sizeof(double) * n);
   int *windows = malloc(sizeof(int) * d);
   for (int i = 0; i < d; i++) windows[i] = i;

   /* which library serves the drop-in name */
   Dl_info info;
   if (dladdr((void *)&Nfft4GPPrecondNysSolve, &info) && info.dli_fname) {
      const char *slash = strrchr(info.dli_fname, '/');
      printf("Nfft4GPPrecondNysSolve from %s\n", slash ? slash + 1 : info.dli_fname);
   }

   /* foo2.cpp:252-267: the dense additive kernel and a precond_nys with a fixed permutation */
   pnfft4gp_kernel kdata =
       (pnfft4gp_kernel)Nfft4GPKernelAdditiveKernelParamCreate(X, n, n, d, windows, d, 1, &Nfft4GPKernelGaussianKernel);
   kdata->_params[0] = f;
   kdata->_params[1] = l;
   kdata->_noise_level = mu;
   double *K = NULL;
   if (Nfft4GPKernelAdditiveKernel(kdata, X, n, n, d, NULL, 0, NULL, 0, &K, NULL) != 0) return 3;
   pprecond_nys nys = (pprecond_nys)Nfft4GPPrecondNysCreate();
   Nfft4GPPrecondNysSetPerm(nys, perm, 0);
   Nfft4GPPrecondNysSetRank(nys, k);
   if (Nfft4GPPrecondNysSetupWithKernel(X, n, n, d, &Nfft4GPKernelAdditiveKernel, kdata, grad, nys) != 0) return 4;

   double *out = calloc((size_t)6 * n + 3, sizeof(double));
   /* the drop-in apply, and the reference's own Solve looked up in its library for an in-process comparison */
   if (Nfft4GPPrecondNysSolve(nys, n, out, rhs) != 0) return 5;
   void *ref = dlopen("libnfft4gp_ref.so", RTLD_NOW | RTLD_NOLOAD);
   func_solve ref_solve = ref ? (func_solve)dlsym(ref, "Nfft4GPPrecondNysSolve") : NULL;
   if (!ref_solve) return 6;
   double *rhs2 = malloc(sizeof(double) * n);
   memcpy(rhs2, rhs, sizeof(double) * n);
   if (ref_solve(nys, n, out + n, rhs2) != 0) return 7;

   /* pcg.c through the drop-in names: the dense operator (host callback) with &Nfft4GPPrecondNysSolve */
   double *x = out + 2 * (size_t)n;
   double rel = 0.0, *relv = NULL;
   int iter = 0;
   nys->_tits = 0;
   if (Nfft4GPSolverPcg(K, n, &Nfft4GPDenseMatSymv, nys, &Nfft4GPPrecondNysSolve, x, b, 1000, 0, 1e-6, &rel, &relv,
                        &iter, 0) != 0)
      return 8;
   out[3 * (size_t)n] = iter;
   out[3 * (size_t)n + 1] = rel;
   out[3 * (size_t)n + 2] = nys->_tits;
   printf("pcg iters %d rel_res %.3e applies %d\n", iter, rel, nys->_tits);
   if (grad) {
      double *y = out + 3 * (size_t)n + 3;
      if (Nfft4GPPrecondNysDvp(nys, n, NULL, rhs, &y) != 0) return 9;
   }
   char path[4096];
   snprintf(path, sizeof path, "%s/out.bin", dir);
   FILE *fo = fopen(path, "wb");
   fwrite(out, sizeof(double), (size_t)6 * n + 3, fo);
   fclose(fo);
   Nfft4GPAmdPrecondNysMirrorRelease(nys);
   Nfft4GPPrecondNysFree(nys);
   printf("DONE\n");
   return 0;
}
