/* struct_offsets.c -- offsetof / sizeof of every field of nfft4gp_kernel (SRC/linearalg/kernels.h:65-95),
 * str_adj (INC/_external.h:28-51) and precond_nys (SRC/preconds/nys.h:24-55).  Compiled twice by tests/test_dropin.py: once against the reference's
 * own declarations (-DUSE_REF, /root/reference in this container) and once against include/nfft4gp_amd.h;
 * the two outputs must be identical. */
#include <stddef.h>
#include <stdio.h>
#ifdef USE_REF
#include "kernels.h" /* SRC/linearalg */
/* str_adj as INC/_external.h:28-51 declares it: that header needs NFFT3's fastsum.h (absent), so the test
 * extracts the struct's text from it into a scratch ref_str_adj.h at run time */
typedef struct fastsum_plan_ fastsum_plan;
#include "ref_str_adj.h"
#include "nys.h" /* SRC/preconds */
#else
#include "nfft4gp_amd.h"
#endif

#define F(T, f) printf("%s.%s %zu %zu\n", #T, #f, offsetof(T, f), sizeof(((T *)0)->f))
int main(void)
{
   printf("nfft4gp_kernel %zu\n", sizeof(nfft4gp_kernel));
   F(nfft4gp_kernel, _params);
   F(nfft4gp_kernel, _iparams);
   F(nfft4gp_kernel, _max_n);
   F(nfft4gp_kernel, _omp);
   F(nfft4gp_kernel, _noise_level);
   F(nfft4gp_kernel, _own_buffer);
   F(nfft4gp_kernel, _buffer);
   F(nfft4gp_kernel, _own_dbuffer);
   F(nfft4gp_kernel, _dbuffer);
   F(nfft4gp_kernel, _fkernel_buffer);
   F(nfft4gp_kernel, _ibufferp);
   F(nfft4gp_kernel, _libufferp);
   F(nfft4gp_kernel, _own_fkernel_buffer_params);
   F(nfft4gp_kernel, _fkernel_buffer_params);
   F(nfft4gp_kernel, _ldwork);
   F(nfft4gp_kernel, _dwork);
   F(nfft4gp_kernel, _external);
   printf("str_adj %zu\n", sizeof(str_adj));
   F(str_adj, _kernel);
   F(str_adj, _d);
   F(str_adj, _sigma);
   F(str_adj, _mu);
   F(str_adj, _N);
   F(str_adj, _p);
   F(str_adj, _m);
   F(str_adj, _eps);
   F(str_adj, _n);
   F(str_adj, _NN);
   F(str_adj, _x);
   F(str_adj, _scale);
   F(str_adj, _kernel_scale);
   F(str_adj, _fastsum_original);
   F(str_adj, _fastsum_derivative);
   printf("precond_nys %zu\n", sizeof(precond_nys));
   F(precond_nys, _k_setup);
   F(precond_nys, _own_perm);
   F(precond_nys, _perm);
   F(precond_nys, _n);
   F(precond_nys, _tits);
   F(precond_nys, _titt);
   F(precond_nys, _tset);
   F(precond_nys, _tlogdet);
   F(precond_nys, _tdvp);
   F(precond_nys, _nys_opt);
   F(precond_nys, _k);
   F(precond_nys, _eta);
   F(precond_nys, _f2);
   F(precond_nys, _U);
   F(precond_nys, _s);
   F(precond_nys, _work);
   F(precond_nys, _K);
   F(precond_nys, _dU);
   F(precond_nys, _dK);
   F(precond_nys, _chol_K11);
   F(precond_nys, _dvp_nosolve);
   return 0;
}
