// stats.hip -- output analysis on the device: effective sample size of every (chain, parameter)
// series of a batched MCMCChain (src/stats/ess.jl:6-10, var.jl:7-8,20-27,45-117).
//
// One thread owns one series x_t = samples[t][j][c] (t < n kept steps): the C-ABI sample layout
// [nkept][d][C] makes a wave's 64 series (consecutive chains c, one parameter j) one coalesced
// 512 B row per t.  The series is staged in LDS ([n][64] doubles) when it fits, otherwise re-read
// from global memory (L2) per lag.  Geyer's sequences need only the lags up to the first
// non-positive pair sum, so the autocovariances are computed lazily, lag pair by lag pair.
//
// Arithmetic order (restated bit for bit by oracle/oracle.c orc_ess): sums left to right over t,
// plain multiply-then-add (no fma), as Julia's var/acf loops.
#include "../common.hpp"
#include "../host/kernels_api.hpp"

namespace mcmc {

constexpr int kEssBlock = 64;

struct EssArgs {
    const double* s;
    int64_t n, d, C;
    int64_t maxlag;
    int64_t batchlen;
    int32_t vtype;        // 1 imse, 2 ipse, 3 bm
    double* ess;          // [d][C]
    double* var;          // [d][C] or NULL: the vtype variance of the mean
};

template <bool LDS>
struct Series {
    const double* col;    // &samples[0][j][c]
    size_t stride;        // d * C
    const double* lds;    // [n][64] (LDS) column of this thread
    __device__ __forceinline__ double x(int64_t t) const {
        return LDS ? lds[(size_t)t * kEssBlock] : col[(size_t)t * stride];
    }
};

template <bool LDS>
__global__ __launch_bounds__(kEssBlock) void k_ess(EssArgs a) {
    extern __shared__ double stage[];
    const int64_t c = (int64_t)blockIdx.x * kEssBlock + threadIdx.x;
    const int64_t j = blockIdx.y;
    const bool live = c < a.C;
    const int64_t n = a.n;
    Series<LDS> S;
    S.stride = (size_t)a.d * (size_t)a.C;
    S.col = a.s + (size_t)j * (size_t)a.C + (size_t)(live ? c : 0);
    S.lds = stage + threadIdx.x;
    // mean (mean.jl:6): left to right.  Rows are loaded 8 at a time so that 8 coalesced 512 B loads
    // per wave are in flight (the staging pass is latency-bound otherwise: few waves fit beside the
    // [n][64] LDS image).
    double sum = 0.0;
    int64_t t = 0;
    for (; t + 8 <= n; t += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = S.col[(size_t)(t + u) * S.stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (LDS) stage[(size_t)(t + u) * kEssBlock + threadIdx.x] = v[u];
            sum = sum + v[u];
        }
    }
    for (; t < n; ++t) {
        const double v = S.col[(size_t)t * S.stride];
        if (LDS) stage[(size_t)t * kEssBlock + threadIdx.x] = v;
        sum = sum + v;
    }
    const double nd = (double)n;
    const double mean = sum / nd;
    // sum of squares of the centred series: var(x) = ss/(n-1) (var.jl:7-8), acv[0] = ss/n
    double ss = 0.0;
    for (int64_t t = 0; t < n; ++t) {
        const double z = S.x(t) - mean;
        ss = ss + z * z;
    }
    const double var_iid = (ss / (nd - 1.0)) / nd;
    double var_v;
    if (a.vtype == 3) {
        // batch means (var.jl:20-27): batchlen * var(batch means) / (nbatches * batchlen)
        const int64_t bl = a.batchlen;
        const int64_t nb = n / bl;
        double bsum = 0.0;
        for (int64_t b = 0; b < nb; ++b) {
            double s = 0.0;
            for (int64_t t = b * bl; t < (b + 1) * bl; ++t) s = s + S.x(t);
            bsum = bsum + s / (double)bl;
        }
        const double bmean = bsum / (double)nb;
        double bss = 0.0;
        for (int64_t b = 0; b < nb; ++b) {
            double s = 0.0;
            for (int64_t t = b * bl; t < (b + 1) * bl; ++t) s = s + S.x(t);
            const double e = s / (double)bl - bmean;
            bss = bss + e * e;
        }
        var_v = ((double)bl * (bss / (double)(nb - 1))) / (double)(nb * bl);
    } else {
        // Geyer's initial monotone (imse, var.jl:45-75) / positive (ipse, var.jl:95-117) sequence:
        // g_j = acv[2j] + acv[2j+1] for j = 0..k, k = floor((maxlag-1)/2), stopping at the first g_j <= 0
        const int64_t maxlag = a.maxlag;
        const int64_t k = (maxlag - 1) >= 0 ? (maxlag - 1) / 2 : -1;
        const double acv0 = ss / nd;
        double gsum = 0.0, prev = 0.0;
        for (int64_t jj = 0; jj <= k; ++jj) {
            double acv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t lag = 2 * jj + h;
                if (lag == 0) {
                    acv[h] = acv0;
                    continue;
                }
                double s = 0.0;                                   // acf(x, lag, correlation=false)
                for (int64_t t = 0; t + lag < n; ++t) s = s + (S.x(t) - mean) * (S.x(t + lag) - mean);
                acv[h] = s / nd;
            }
            double g = acv[0] + acv[1];
            if (g <= 0.0) break;                                  // m = j
            if (a.vtype == 1 && jj > 0 && g > prev) g = prev;     // monotone: g[j] = min(g[j], g[j-1])
            prev = g;
            gsum = gsum + g;
        }
        var_v = (-acv0 + 2.0 * gsum) / nd;
    }
    if (live) {
        const size_t o = (size_t)j * (size_t)a.C + (size_t)c;
        a.ess[o] = (nd * var_iid) / var_v;                        // ess.jl:9
        if (a.var) a.var[o] = var_v;
    }
}

}  // namespace mcmc

hipError_t mcmc_launch_ess(const double* samples, int64_t n, int64_t d, int64_t C, int32_t vtype, int64_t maxlag,
                           int64_t batchlen, double* ess, double* var, hipStream_t st) {
    using namespace mcmc;
    EssArgs a{samples, n, d, C, maxlag, batchlen, vtype, ess, var};
    const dim3 grid((unsigned)((C + kEssBlock - 1) / kEssBlock), (unsigned)d);
    const size_t lds = (size_t)n * kEssBlock * sizeof(double);
    if (lds <= 64 * 1024)
        k_ess<true><<<grid, kEssBlock, lds, st>>>(a);
    else
        k_ess<false><<<grid, kEssBlock, 0, st>>>(a);
    return hipGetLastError();
}
