// window.cpp -- host-side NFFT window, kernel Fourier coefficients and tap polynomials.
//
// Follows the algorithm NFFT3's fastsum (third-party, called from nfft_interface.c:227-254 and
// :426) applies with the reference's hard-coded parameters N = 32, n_os = 64, m = 4, p = 1,
// eps_I = eps_B = 0 (nfft_interface.c:18-27):
//   * Kaiser-Bessel window PHI / PHI_HUT with b = pi (2 - 1/sigma), sigma = 2;
//   * bhat_k = N^-1 sum_{l=-N/2}^{N/2-1} K(|l|/N) e^{-2 pi i k l / N} (real: K is even);
//   * the spread -> FFT -> /phihut -> *bhat -> /phihut -> IFFT -> interpolate chain, whose middle
//     part (everything between spreading and interpolation) is, on the real part the reference
//     keeps (nfft_interface.c:436), the circulant
//       w[s] = sum_{k=-N/2}^{N/2-1} bhat_k / phihut_k^2 cos(2 pi k s / n_os).
#include <cmath>
#include <complex>
#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "internal.h"

namespace nfft4gp_amd {

static const double kPi = 3.141592653589793238462643383279502884;

static double kb_b() { return kPi * (2.0 - 1.0 / ((double)kNos / (double)kBand)); }

double kb_phi(double t)
{
   const double b = kb_b();
   const double a = (double)(kM * kM) - t * t;
   if (a > 0.0) {
      const double s = std::sqrt(a);
      return std::sinh(b * s) / (kPi * s);
   }
   if (a < 0.0) {
      const double s = std::sqrt(-a);
      return std::sin(b * s) / (kPi * s);
   }
   return b / kPi;
}

static double bessel_i0(double z)
{
   double sum = 1.0, term = 1.0;
   const double q = 0.25 * z * z;
   for (int k = 1; k < 200; k++) {
      term *= q / ((double)k * (double)k);
      sum += term;
      if (term < 1e-18 * sum) break;
   }
   return sum;
}

double kb_phi_hut(int k)
{
   const double b = kb_b();
   const double w = 2.0 * kPi * (double)k / (double)kNos;
   return bessel_i0((double)kM * std::sqrt(b * b - w * w));
}

// Chebyshev interpolation of each tap on u in [-1/2, 1/2] at kNC nodes, converted to monomials in
// u with long-double arithmetic.  Tap t of a point at offset frac in its cell is PHI(frac + m - t).
static std::vector<double> fit_taps()
{
   std::vector<double> C(kTaps * kNC, 0.0);
   const int n = kNC;
   for (int t = 0; t < kTaps; t++) {
      // Chebyshev coefficients a_j of g(z) = tap(u = z/2), z in [-1, 1]
      std::vector<long double> fz(n), a(n, 0.0L);
      for (int i = 0; i < n; i++) {
         const long double z = std::cos(kPi * (i + 0.5) / n);
         fz[i] = (long double)kb_phi((double)(z / 2.0L) + 0.5 + kM - t);
      }
      for (int j = 0; j < n; j++) {
         long double s = 0.0L;
         for (int i = 0; i < n; i++) s += fz[i] * std::cos((long double)kPi * j * (i + 0.5L) / n);
         a[j] = s * (j == 0 ? 1.0L : 2.0L) / n;
      }
      // T_j(z) -> monomials in z by the three-term recurrence
      std::vector<std::vector<long double>> T(n, std::vector<long double>(n, 0.0L));
      T[0][0] = 1.0L;
      if (n > 1) T[1][1] = 1.0L;
      for (int j = 2; j < n; j++)
         for (int p = 0; p < n; p++)
            T[j][p] = (p > 0 ? 2.0L * T[j - 1][p - 1] : 0.0L) - T[j - 2][p];
      for (int p = 0; p < n; p++) {
         long double c = 0.0L;
         for (int j = 0; j < n; j++) c += a[j] * T[j][p];
         // z = 2u  ->  z^p = 2^p u^p
         C[t * kNC + p] = (double)(c * std::pow(2.0L, (long double)p));
      }
   }
   return C;
}

const std::vector<double>& tap_poly_coeffs()
{
   static std::once_flag once;
   static std::vector<double> C;
   std::call_once(once, [] { C = fit_taps(); });
   return C;
}

static double kern(int kind, double r, double c)
{
   r = std::fabs(r);
   switch (kind) {
   case 0: return std::exp(-r * r / (c * c));                      // gaussian
   case 1: return (r * r / (c * c)) * std::exp(-r * r / (c * c));  // xx_gaussian
   case 2: return std::exp(-r / c);                                // laplacian_rbf
   case 3: return (r / c) * std::exp(-r / c);                      // der_laplacian_rbf
   }
   return 0.0;
}

void bhat_1d(int kind, double c, double* bhat)
{
   const int N = kBand;
   double s[kBand];
   for (int l = 0; l < N; l++) {
      double r = (double)(l - N / 2) / (double)N;
      if (std::fabs(r) > 0.5) r = 0.5;
      s[l] = kern(kind, r, c) / (double)N;
   }
   for (int k = 0; k < N; k++) {
      double acc = 0.0;
      for (int l = 0; l < N; l++) {
         const long long ph = (long long)(k - N / 2) * (long long)(l - N / 2);
         const int m = (int)(((ph % N) + N) % N);  // exact phase reduction
         acc += s[l] * std::cos(2.0 * kPi * (double)m / (double)N);
      }
      bhat[k] = acc;
   }
}

// d-dimensional bhat on the N^d modes (index sum_t (k_t + N/2) N^t): the N^-d scaled samples
// K(min(|l/N|, 1/2)) transformed one axis at a time in complex arithmetic, real part kept (the
// imaginary part cancels: the samples are even apart from the unpaired l_t = -N/2 planes, whose
// phase factors are +-1)
void bhat_nd(int kind, int d, double c, std::vector<double>& bhat)
{
   const int N = kBand;
   int nm = 1;
   for (int t = 0; t < d; t++) nm *= N;
   std::vector<std::complex<double>> a(nm), b(nm);
   for (int j = 0; j < nm; j++) {
      int jj = j;
      double r2 = 0.0;
      for (int t = 0; t < d; t++) {
         const double lt = (double)(jj % N - N / 2) / (double)N;
         r2 += lt * lt;
         jj /= N;
      }
      double r = std::sqrt(r2);
      if (r > 0.5) r = 0.5;
      a[j] = kern(kind, r, c) / (double)nm;
   }
   std::complex<double> tw[kBand];
   for (int m = 0; m < N; m++) tw[m] = std::polar(1.0, -2.0 * kPi * (double)m / (double)N);
   // 5-feature windows have 32^5 modes (5 passes of 1.1e9 complex products): the passes are split over up to
   // 16 host threads by output index (each output's sum is unchanged, so are the bits)
   const int nth = nm >= (1 << 20) ? std::max(1, std::min(16, (int)std::thread::hardware_concurrency())) : 1;
   int stride = 1;
   for (int t = 0; t < d; t++) {
      auto pass = [&](int j0, int j1) {
         for (int j = j0; j < j1; j++) {
            const int lo = j % stride, kt = (j / stride) % N, hi = j / (stride * N);
            std::complex<double> acc = 0.0;
            for (int l = 0; l < N; l++) {
               const int m = ((((kt - N / 2) * (l - N / 2)) % N) + N) % N;  // exact phase reduction
               acc += a[lo + stride * (l + N * hi)] * tw[m];
            }
            b[j] = acc;
         }
      };
      if (nth == 1) {
         pass(0, nm);
      } else {
         std::vector<std::thread> th;
         const int per = (nm + nth - 1) / nth;
         for (int i = 0; i < nth; i++) th.emplace_back(pass, std::min(nm, i * per), std::min(nm, (i + 1) * per));
         for (auto& x : th) x.join();
      }
      a.swap(b);
      stride *= N;
   }
   bhat.resize(nm);
   for (int j = 0; j < nm; j++) bhat[j] = a[j].real();
}

void circulant_1d(const double* bhat, double weight, double* w)
{
   const int N = kBand;
   double coef[kBand];
   for (int k = 0; k < N; k++) {
      const double ph = kb_phi_hut(k - N / 2);
      coef[k] = bhat[k] / (ph * ph);
   }
   for (int s = 0; s < kNos; s++) {
      double acc = 0.0;
      for (int k = 0; k < N; k++) {
         const int kk = k - N / 2;
         const int m = (((kk * s) % kNos) + kNos) % kNos;
         acc += coef[k] * std::cos(2.0 * kPi * (double)m / (double)kNos);
      }
      w[s] = weight * acc;
   }
}

}  // namespace nfft4gp_amd
