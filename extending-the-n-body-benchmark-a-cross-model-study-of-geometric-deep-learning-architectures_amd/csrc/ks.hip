// Two-sample Kolmogorov-Smirnov statistics of the self-feed macro series on the device
// (utils/ks_utils.py:7-17 `_ks_p`: NaNs dropped, then scipy.stats.ks_2samp's statistic
// D = max_x |F_a(x) - F_b(x)|, with F(x) = #{samples <= x} / n evaluated at every sample,
// i.e. numpy searchsorted(side='right') over the concatenated data).
//
// One workgroup per (a, b) pair.  Both samples are staged into LDS (fp64, NaN and padding
// ordered after every number), bitonic-sorted in place, then every thread takes samples of
// the concatenation, evaluates both empirical CDFs by binary search (upper bound) and the
// block reduces max |F_a - F_b|.  The CDF values are the same k / n fp64 divisions numpy
// performs, so D is bit-exact with scipy's.  The p-value is a scalar function of (D, n_a, n_b)
// computed on the host (ks.py).
#include <cmath>

#include "nbx_internal.h"

namespace {

constexpr int KS_THREADS = 1024;
constexpr int KS_MAX_N = 8192;   // per sample: two [8192] fp64 arrays = 128 KiB of LDS

// total order with NaN last (NaN == NaN)
__device__ __forceinline__ bool ks_less(double x, double y) {
    const bool nx = x != x, ny = y != y;
    if (nx || ny) return !nx && ny;
    return x < y;
}

__device__ void ks_bitonic(double* s, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const double a = s[i], b = s[l];
                    if (up ? ks_less(b, a) : ks_less(a, b)) {
                        s[i] = b;
                        s[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// number of elements <= x among the n sorted numbers s[0..n)
__device__ __forceinline__ int ks_upper(const double* s, int n, double x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(KS_THREADS) void ks_stat_kernel(const double* __restrict__ a, int64_t na, int64_t lda,
                                                             const double* __restrict__ b, int64_t nb, int64_t ldb,
                                                             double* __restrict__ d_out, int64_t* __restrict__ n_out) {
    extern __shared__ double lds[];
    __shared__ int cnt[2];
    __shared__ double red[KS_THREADS / 64];
    const int pair = blockIdx.x;
    const int t = threadIdx.x;
    int Pa = 1, Pb = 1;
    while (Pa < na) Pa <<= 1;
    while (Pb < nb) Pb <<= 1;
    double* sa = lds;
    double* sb = lds + Pa;
    if (t < 2) cnt[t] = 0;
    __syncthreads();
    int va = 0, vb = 0;
    for (int i = t; i < Pa; i += blockDim.x) {
        const double x = i < na ? a[pair * lda + i] : NAN;
        sa[i] = x;
        va += x == x;
    }
    for (int i = t; i < Pb; i += blockDim.x) {
        const double x = i < nb ? b[pair * ldb + i] : NAN;
        sb[i] = x;
        vb += x == x;
    }
    atomicAdd(&cnt[0], va);
    atomicAdd(&cnt[1], vb);
    __syncthreads();
    ks_bitonic(sa, Pa);
    ks_bitonic(sb, Pb);
    const int n1 = cnt[0], n2 = cnt[1];
    double dmax = 0.0;
    if (n1 > 0 && n2 > 0) {
        for (int i = t; i < n1 + n2; i += blockDim.x) {
            const double x = i < n1 ? sa[i] : sb[i - n1];
            const double c1 = (double)ks_upper(sa, n1, x) / (double)n1;
            const double c2 = (double)ks_upper(sb, n2, x) / (double)n2;
            dmax = fmax(dmax, fabs(c1 - c2));
        }
    }
    for (int off = 32; off > 0; off >>= 1) dmax = fmax(dmax, __shfl_xor(dmax, off));
    if ((t & 63) == 0) red[t >> 6] = dmax;
    __syncthreads();
    if (t == 0) {
        double m = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = fmax(m, red[w]);
        d_out[pair] = (n1 > 0 && n2 > 0) ? m : NAN;
        if (n_out) {
            n_out[2 * pair] = n1;
            n_out[2 * pair + 1] = n2;
        }
    }
}

}  // namespace

extern "C" int nbx_ks_2samp_stat(const double* a, int64_t na, int64_t lda, const double* b, int64_t nb, int64_t ldb,
                                 int64_t num_pairs, double* d_out, int64_t* n_out, void* stream) {
    NBX_CHECK_ARG(a && b && d_out && num_pairs >= 0, "nbx_ks_2samp_stat: bad arguments");
    NBX_CHECK_ARG(na >= 1 && nb >= 1 && na <= KS_MAX_N && nb <= KS_MAX_N,
                  "nbx_ks_2samp_stat: sample sizes must be in [1, %d] (got %lld, %lld)", KS_MAX_N, (long long)na,
                  (long long)nb);
    NBX_CHECK_ARG(lda >= na && ldb >= nb, "nbx_ks_2samp_stat: leading dimensions too small");
    if (num_pairs == 0) return NBX_OK;
    int Pa = 1, Pb = 1;
    while (Pa < na) Pa <<= 1;
    while (Pb < nb) Pb <<= 1;
    const size_t shm = sizeof(double) * (size_t)(Pa + Pb);
    hipStream_t st = (hipStream_t)stream;
    if (shm > 64 * 1024) NBX_HIP(hipFuncSetAttribute((const void*)ks_stat_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    hipLaunchKernelGGL(ks_stat_kernel, dim3((unsigned)num_pairs), dim3(KS_THREADS), shm, st, a, na, lda, b, nb, ldb,
                       d_out, n_out);
    NBX_LAUNCH_CHECK("ks_stat");
    return NBX_OK;
}
