// stats.hip -- output analysis on the device: effective sample size of every (chain, parameter)
// series of a batched MCMCChain (src/stats/ess.jl:6-10, var.jl:7-8,20-27,45-117).
//
// The C-ABI sample layout [nkept][d][C] makes 64 consecutive chains of one parameter one coalesced
// 512 B row per kept step t.  k_ess_tile (n up to kEssTileMaxN): a 256-thread block stages the n x 64 tile
// of its 64 series in LDS once; one lane per series sums and centres its series in place (z_t = x_t - mean);
// then four lanes per series compute Geyer's lag pairs four at a time (lane q of round r: the pair
// j = 4r + q, lags 2j and 2j + 1), share the four pair sums, and every lane of the group runs the
// sequential initial-sequence scan on them; the rounds stop at the series' first non-positive pair
// (at most three pairs are computed past it and discarded).  The lag sums read LDS only (no HBM re-reads):
// one read of z_t (broadcast to the group) and one of z_{t+2j+1} per step, two FMAs.  Longer series
// (k_ess_col) keep one thread per series and re-read the column from global memory (L2) per lag.
//
// Arithmetic order (restated bit for bit by oracle/oracle.c orc_ess): the sum of x and every lag sum
// left to right over t; ss and the autocovariance sums accumulate with fma(z_t, z_{t+lag}, s); batch sums
// plain adds.  The lag-0 sum is ss itself (the same fma chain), so acv0 = ss / n.
#include "../common.hpp"
#include "../host/kernels_api.hpp"

namespace mcmc {

constexpr int kEssBlock = 64;          // k_ess_col: one thread per series
constexpr int kEssTile = 64;           // k_ess_tile: series per block
constexpr int kEssThreads = 256;       // k_ess_tile: 4 lanes per series
constexpr int kEssRow = 72;            // LDS row stride in doubles: the 4 lag rows of a lane group (2 rows
                                       // apart) land 32 banks apart, so a wave's 64 reads take the minimum 2 passes
constexpr int kEssTileMaxN = (160 * 1024) / (kEssRow * 8);    // 284: the tile fits the 160 KB of LDS

struct EssArgs {
    const double* s;
    int64_t n, d, C;
    int64_t maxlag;
    int64_t batchlen;
    int32_t vtype;        // 1 imse, 2 ipse, 3 bm
    double* ess;          // [d][C]
    double* var;          // [d][C] or NULL: the vtype variance of the mean
};

// batch means (var.jl:20-27): batchlen * var(batch means) / (nbatches * batchlen); x(t) = the raw series
template <class X>
__device__ __forceinline__ double ess_bm(const X& x, int64_t n, int64_t bl) {
    const int64_t nb = n / bl;
    double bsum = 0.0;
    for (int64_t b = 0; b < nb; ++b) {
        double s = 0.0;
        for (int64_t t = b * bl; t < (b + 1) * bl; ++t) s = s + x(t);
        bsum = bsum + s / (double)bl;
    }
    const double bmean = bsum / (double)nb;
    double bss = 0.0;
    for (int64_t b = 0; b < nb; ++b) {
        double s = 0.0;
        for (int64_t t = b * bl; t < (b + 1) * bl; ++t) s = s + x(t);
        const double e = s / (double)bl - bmean;
        bss = bss + e * e;
    }
    return ((double)bl * (bss / (double)(nb - 1))) / (double)(nb * bl);
}

// Geyer's initial sequence step for pair j with pair sum g (var.jl:45-75 imse, :95-117 ipse); returns
// false at the first non-positive pair (m = j) -- the sequence ends there
__device__ __forceinline__ bool geyer_take(double g, int64_t j, int32_t vtype, double& prev, double& gsum) {
    if (g <= 0.0) return false;
    if (vtype == 1 && j > 0 && g > prev) g = prev;             // monotone: g[j] = min(g[j], g[j-1])
    prev = g;
    gsum = gsum + g;
    return true;
}

__global__ __launch_bounds__(kEssThreads) void k_ess_tile(EssArgs a) {
    extern __shared__ double tile[];                           // [n][kEssRow]: x, then z = x - mean
    const int tid = (int)threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * kEssTile;
    const int64_t j = blockIdx.y;
    const int64_t n = a.n;
    const size_t stride = (size_t)a.d * (size_t)a.C;
    const double* base = a.s + (size_t)j * (size_t)a.C;
    // stage: 4 rows per pass of the block, 8 passes in flight
    {
        const int cc = tid & 63;
        const bool live = c0 + cc < a.C;
        const double* col = base + (size_t)(live ? c0 + cc : 0);
        int64_t t = tid >> 6;
        for (; t + 28 < n; t += 32) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = col[(size_t)(t + 4 * u) * stride];
#pragma unroll
            for (int u = 0; u < 8; ++u) tile[(size_t)(t + 4 * u) * kEssRow + cc] = live ? v[u] : 0.0;
        }
        for (; t < n; t += 4) tile[(size_t)t * kEssRow + cc] = live ? col[(size_t)t * stride] : 0.0;
    }
    __syncthreads();
    const int sr = tid >> 2, q = tid & 3;                      // series (column) and lane within its group
    double* zc = tile + sr;
    const double nd = (double)n;
    double ss = 0.0, var_v = 0.0;
    if (q == 0) {
        double sum = 0.0;                                      // mean (mean.jl:6), left to right
        for (int64_t t = 0; t < n; ++t) sum = sum + zc[(size_t)t * kEssRow];
        const double mean = sum / nd;
        if (a.vtype == 3) var_v = ess_bm([&](int64_t t) { return zc[(size_t)t * kEssRow]; }, n, a.batchlen);
        for (int64_t t = 0; t < n; ++t) {
            const double z = zc[(size_t)t * kEssRow] - mean;
            zc[(size_t)t * kEssRow] = z;
            ss = __builtin_fma(z, z, ss);
        }
    }
    __syncthreads();
    const int gl = (tid & 63) & ~3;                            // the group's first lane in the wave
    ss = __shfl(ss, gl, 64);
    const double acv0 = ss / nd;
    if (a.vtype != 3) {
        const int64_t k = (a.maxlag - 1) >= 0 ? (a.maxlag - 1) / 2 : -1;
        double gsum = 0.0, prev = 0.0;
        bool done = k < 0;
        for (int64_t r0 = 0; !__all(done); r0 += 4) {
            const int64_t jp = r0 + q;                         // this lane's pair
            double g = 0.0;
            if (!done && jp <= k) {
                const int64_t L0 = 2 * jp, L1 = L0 + 1;        // lags; L1 <= maxlag <= n - 1
                double s0 = 0.0, s1 = 0.0;
                double b = zc[(size_t)L0 * kEssRow];           // z_{t+L0}
                for (int64_t t = 0; t + L1 < n; ++t) {
                    const double zt = zc[(size_t)t * kEssRow];
                    const double b1 = zc[(size_t)(t + L1) * kEssRow];
                    s0 = __builtin_fma(zt, b, s0);
                    s1 = __builtin_fma(zt, b1, s1);
                    b = b1;
                }
                s0 = __builtin_fma(zc[(size_t)(n - 1 - L0) * kEssRow], b, s0);   // lag L0's last term
                g = s0 / nd + s1 / nd;                         // acv[2j] + acv[2j+1] (acv[0] = ss/n: the same sum)
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double gi = __shfl(g, gl + i, 64);
                if (!done) done = r0 + i > k || !geyer_take(gi, r0 + i, a.vtype, prev, gsum);
            }
        }
        var_v = (-acv0 + 2.0 * gsum) / nd;
    } else {
        var_v = __shfl(var_v, gl, 64);
    }
    const int64_t c = c0 + sr;
    if (q == 0 && c < a.C) {
        const double var_iid = (ss / (nd - 1.0)) / nd;
        const size_t o = (size_t)j * (size_t)a.C + (size_t)c;
        a.ess[o] = (nd * var_iid) / var_v;                     // ess.jl:9
        if (a.var) a.var[o] = var_v;
    }
}

// long series (n > kEssTileMaxN): one thread per series, the column re-read from global memory per lag
__global__ __launch_bounds__(kEssBlock) void k_ess_col(EssArgs a) {
    const int64_t c = (int64_t)blockIdx.x * kEssBlock + threadIdx.x;
    const int64_t j = blockIdx.y;
    const bool live = c < a.C;
    const int64_t n = a.n;
    const size_t stride = (size_t)a.d * (size_t)a.C;
    const double* col = a.s + (size_t)j * (size_t)a.C + (size_t)(live ? c : 0);
    auto x = [&](int64_t t) { return col[(size_t)t * stride]; };
    double sum = 0.0;
    for (int64_t t = 0; t < n; ++t) sum = sum + x(t);
    const double nd = (double)n;
    const double mean = sum / nd;
    double ss = 0.0;
    for (int64_t t = 0; t < n; ++t) {
        const double z = x(t) - mean;
        ss = __builtin_fma(z, z, ss);
    }
    double var_v;
    if (a.vtype == 3) {
        var_v = ess_bm(x, n, a.batchlen);
    } else {
        const int64_t k = (a.maxlag - 1) >= 0 ? (a.maxlag - 1) / 2 : -1;
        double gsum = 0.0, prev = 0.0;
        for (int64_t jj = 0; jj <= k; ++jj) {
            const int64_t L0 = 2 * jj, L1 = L0 + 1;
            double s0 = 0.0, s1 = 0.0;
            for (int64_t t = 0; t + L1 < n; ++t) {
                const double zt = x(t) - mean;
                s0 = __builtin_fma(zt, x(t + L0) - mean, s0);
                s1 = __builtin_fma(zt, x(t + L1) - mean, s1);
            }
            s0 = __builtin_fma(x(n - 1 - L0) - mean, x(n - 1) - mean, s0);
            if (!geyer_take(s0 / nd + s1 / nd, jj, a.vtype, prev, gsum)) break;
        }
        var_v = (-(ss / nd) + 2.0 * gsum) / nd;
    }
    if (live) {
        const double var_iid = (ss / (nd - 1.0)) / nd;
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
    if (n <= kEssTileMaxN) {
        const size_t lds = (size_t)n * kEssRow * sizeof(double);
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void*)k_ess_tile, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds);
            if (e != hipSuccess) return e;
        }
        const dim3 grid((unsigned)((C + kEssTile - 1) / kEssTile), (unsigned)d);
        k_ess_tile<<<grid, kEssThreads, lds, st>>>(a);
    } else {
        const dim3 grid((unsigned)((C + kEssBlock - 1) / kEssBlock), (unsigned)d);
        k_ess_col<<<grid, kEssBlock, 0, st>>>(a);
    }
    return hipGetLastError();
}
