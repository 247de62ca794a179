// probe: does rocSOLVER from /opt/rocm work inside a process that already loaded PyTorch's ROCm libs?
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <cstdio>

extern "C" int probe_syevd(const double* A_host, int n, double* w_host, double* V_host)
{
   rocblas_handle h;
   if (rocblas_create_handle(&h) != rocblas_status_success) return -1;
   double *dA, *dW, *dE;
   rocblas_int* dinfo;
   hipMalloc(&dA, sizeof(double) * n * n);
   hipMalloc(&dW, sizeof(double) * n);
   hipMalloc(&dE, sizeof(double) * n);
   hipMalloc(&dinfo, sizeof(rocblas_int));
   hipMemcpy(dA, A_host, sizeof(double) * n * n, hipMemcpyHostToDevice);
   rocblas_status st = rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, n, dA, n, dW, dE, dinfo);
   hipDeviceSynchronize();
   rocblas_int info = -1;
   hipMemcpy(&info, dinfo, sizeof(info), hipMemcpyDeviceToHost);
   hipMemcpy(w_host, dW, sizeof(double) * n, hipMemcpyDeviceToHost);
   hipMemcpy(V_host, dA, sizeof(double) * n * n, hipMemcpyDeviceToHost);
   hipFree(dA); hipFree(dW); hipFree(dE); hipFree(dinfo);
   rocblas_destroy_handle(h);
   return st == rocblas_status_success ? (int)info : -100 - (int)st;
}
