// stats.hip -- output analysis on the device: effective sample size of every (chain, parameter)
// series of a batched MCMCChain (src/stats/ess.jl:6-10, var.jl:7-8,20-27,45-117).
//
// The C-ABI sample layout [nkept][d][C] makes consecutive chains of one parameter one coalesced row per kept
// step t.  k_ess_tile (n up to kEssTileMaxN): a 128-thread block stages the n x 32 tile of its 32 series in LDS
// once, series-major (plus a zero pad); one lane per series sums and centres its series in place (z_t = x_t - mean);
// then four lanes per series compute Geyer's lag pairs, first one pair per lane (pairs 0-3: a series of nearly
// independent draws stops there), then four consecutive pairs (eight lags) per lane per round, sixteen pairs
// per series and round.  A lane keeps its eight shifted values in a register window, so each step of its lag
// sums costs one ds_read_b128 per two steps and eight FMAs per step.  The group shares the pair sums and every lane of it runs the
// sequential initial-sequence scan on them; pairs computed past the series' first non-positive pair are
// discarded.  No HBM re-reads.  Longer series (k_ess_col) keep one thread per series and re-read the column
// from global memory (L2) per lag.
//
// Arithmetic order (restated bit for bit by oracle/oracle.c orc_ess): the sum of x and every lag sum
// left to right over t; ss and the autocovariance sums accumulate with fma(z_t, z_{t+lag}, s); batch sums
// plain adds.  The lag-0 sum is ss itself (the same fma chain), so acv0 = ss / n.
#include "../common.hpp"
#include "../host/kernels_api.hpp"

namespace mcmc {

constexpr int kEssBlock = 64;          // k_ess_col: one thread per series
constexpr int kEssTile = 32;           // k_ess_tile: series per block
constexpr int kEssThreads = 128;       // k_ess_tile: 4 lanes per series
// k_ess_tile's LDS tile is series-major, [32][S] doubles: a series is contiguous in t, so two consecutive steps
// come in one ds_read_b128.  S >= n + 16 (a zero pad: the lag loops run in whole 8-step blocks and read up to 15
// past the series' end) and S = 2 mod 8: the 16 lanes of a ds_read_b128 lane group (4 series x 4 lanes whose
// windows sit 8 steps apart) then cover the 64 banks once.
__host__ __device__ constexpr int ess_stride(int n) { return n + 16 + (((2 - (n + 16)) % 8) + 8) % 8; }
constexpr int kEssTileMaxN = 618;      // 32 x ess_stride(618) x 8 B = 162 304 B: fits the 160 KB of LDS
static_assert(32 * ess_stride(kEssTileMaxN) * 8 <= 160 * 1024 && 32 * ess_stride(kEssTileMaxN + 1) * 8 > 160 * 1024,
              "kEssTileMaxN is the largest series the LDS tile holds");

typedef double ess_f64x2 __attribute__((ext_vector_type(2)));

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

// acc[i] = sum over t < tn (tn a multiple of LPL) of z_t z_{t+L0+i}, in t order: lag L0+i's autocovariance sum
// once the zero pad has absorbed the terms past the series' end (fma(z, 0, s) = s; s is never -0).  The LPL
// values z_{t+L0} .. z_{t+L0+LPL-1} ride in a register window rotated by renaming; every two steps take one
// ds_read_b128 of (z_t, z_{t+1}) (shared by the lane group) and one of the window's next two entries.
template <int LPL>
__device__ __forceinline__ void ess_lag_sums(const double* zc, int L0, int tn, double (&acc)[LPL]) {
    double w[LPL];
#pragma unroll
    for (int i = 0; i < LPL; i += 2) {
        const ess_f64x2 v = *reinterpret_cast<const ess_f64x2*>(zc + L0 + i);
        w[i] = v.x;
        w[i + 1] = v.y;
    }
#pragma unroll
    for (int i = 0; i < LPL; ++i) acc[i] = 0.0;
    for (int t = 0; t < tn; t += LPL) {
#pragma unroll
        for (int u = 0; u < LPL; u += 2) {
            const ess_f64x2 zz = *reinterpret_cast<const ess_f64x2*>(zc + t + u);            // z_{t+u}, z_{t+u+1}
            const ess_f64x2 nw = *reinterpret_cast<const ess_f64x2*>(zc + t + u + L0 + LPL); // next window pair
#pragma unroll
            for (int i = 0; i < LPL; ++i) acc[i] = __builtin_fma(zz.x, w[(i + u) % LPL], acc[i]);
            w[u] = nw.x;                                                                     // z_{t+u+L0+LPL}
#pragma unroll
            for (int i = 0; i < LPL; ++i) acc[i] = __builtin_fma(zz.y, w[(i + u + 1) % LPL], acc[i]);
            w[u + 1] = nw.y;
        }
    }
}

// one Geyer round: lane q of the group computes pairs p0 + q LPL/2 ... (lags 2 p0 + q LPL ...), the group's
// 4 LPL/2 pair sums are shared and scanned in pair order by every lane of the group
template <int LPL>
__device__ __forceinline__ void ess_round(const double* zc, int n, double nd, int64_t p0, int q, int gl, int64_t k,
                                          int32_t vtype, bool& done, double& prev, double& gsum) {
    constexpr int PP = LPL / 2;                                // pairs per lane
    double g[PP];
#pragma unroll
    for (int i = 0; i < PP; ++i) g[i] = 0.0;
    const int64_t L0 = 2 * (p0 + (int64_t)q * PP);
    if (!done && p0 + (int64_t)q * PP <= k && L0 < n) {
        double acc[LPL];
        const int tn = (int)((n - L0 + LPL - 1) / LPL) * LPL;
        ess_lag_sums<LPL>(zc, (int)L0, tn, acc);
#pragma unroll
        for (int i = 0; i < PP; ++i) g[i] = acc[2 * i] / nd + acc[2 * i + 1] / nd;   // acv[2j] + acv[2j+1]
    }
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int i = 0; i < PP; ++i) {
            const double gi = __shfl(g[i], gl + qq, 64);
            const int64_t jp = p0 + qq * PP + i;
            if (!done) done = jp > k || !geyer_take(gi, jp, vtype, prev, gsum);
        }
}

__global__ __launch_bounds__(kEssThreads) void k_ess_tile(EssArgs a) {
    extern __shared__ __attribute__((aligned(16))) double tile[];   // [32][S]: x, then z = x - mean, zero pad
    const int tid = (int)threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * kEssTile;
    const int64_t j = blockIdx.y;
    const int n = (int)a.n;
    const int S = ess_stride(n);
    const size_t stride = (size_t)a.d * (size_t)a.C;
    const double* base = a.s + (size_t)j * (size_t)a.C;
    // stage: rows of 32 chains (256 B) from HBM, 4 rows per pass of the block, transposed into the series-major
    // tile; then the zero pad
    {
        const int cc = tid & 31;
        const bool live = c0 + cc < a.C;
        const double* col = base + (size_t)(live ? c0 + cc : 0);
        double* dst = tile + cc * S;
        // every row of a 96-row pass requested before the first is written to LDS (24 loads in flight per thread:
        // the staging is latency-bound otherwise, a block's whole tile being one HBM round trip)
        for (int t0 = tid >> 5; t0 < n; t0 += 96) {
            double v[24];
#pragma unroll
            for (int u = 0; u < 24; ++u) {
                const int t = t0 + 4 * u;
                v[u] = (live && t < n) ? col[(size_t)t * stride] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 24; ++u)
                if (t0 + 4 * u < n) dst[t0 + 4 * u] = v[u];
        }
        for (int t2 = n + (tid >> 5); t2 < S; t2 += 4) dst[t2] = 0.0;
    }
    __syncthreads();
    const int sr = tid >> 2, q = tid & 3;                      // series and lane within its group
    double* zc = tile + sr * S;
    const double nd = (double)n;
    double ss = 0.0, var_v = 0.0;
    if (q == 0) {
        // mean (mean.jl:6), left to right; 16 steps of LDS reads in flight per block of the dependent adds
        double sum = 0.0;
        int t = 0;
        for (; t + 16 <= n; t += 16) {
            ess_f64x2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const ess_f64x2*>(zc + t + 2 * u);
#pragma unroll
            for (int u = 0; u < 8; ++u) sum = (sum + v[u].x) + v[u].y;
        }
        for (; t < n; ++t) sum = sum + zc[t];
        const double mean = sum / nd;
        if (a.vtype == 3) var_v = ess_bm([&](int64_t t) { return zc[t]; }, (int64_t)n, a.batchlen);
        // centre in place; ss = sum of z^2 with the lag sums' fma chain
        for (t = 0; t + 16 <= n; t += 16) {
            ess_f64x2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const ess_f64x2*>(zc + t + 2 * u);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                v[u].x = v[u].x - mean;
                v[u].y = v[u].y - mean;
                ss = __builtin_fma(v[u].x, v[u].x, ss);
                ss = __builtin_fma(v[u].y, v[u].y, ss);
                *reinterpret_cast<ess_f64x2*>(zc + t + 2 * u) = v[u];
            }
        }
        for (; t < n; ++t) {
            const double z = zc[t] - mean;
            zc[t] = z;
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
        // round 0: one pair per lane (pairs 0-3; nearly independent draws stop there), then 4 pairs per lane
        ess_round<2>(zc, n, nd, 0, q, gl, k, a.vtype, done, prev, gsum);
        for (int64_t p0 = 4; !__all(done); p0 += 16) ess_round<8>(zc, n, nd, p0, q, gl, k, a.vtype, done, prev, gsum);
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

// Series of up to N = 32, 64 or 96 kept samples, IMSE/IPSE (the metric keeps 90): one lane per series, the whole
// series in registers.  A wave covers 64 consecutive chains of one parameter, so every load of a step is one
// coalesced 512-byte row; no LDS, no staging round trip, no cross-lane traffic: the mean, the centring and the
// sums of squares run on every lane, and each lane scans its own pairs.  Lag sums go two pairs (four lags, four
// independent fma chains) per step; the wave leaves the unrolled pair loop once all its series have met their
// first non-positive pair (or k), so a wave pays for its slowest series only -- against k_ess_tile's fixed rounds of
// sixteen pairs.  N - 32 < n <= N (N = 32: 2 <= n <= 32): positions t >= n hold exact zeros, which leave every sum
// unchanged (s + 0 = s and fma(z, 0, s) = s, s never being -0), so the arithmetic is k_ess_tile's (and orc_ess's)
// bit for bit: left-to-right sum, ss and every lag sum an fma chain in t order.
template <int N>
__global__ __launch_bounds__(256, 2) void k_ess_reg(EssArgs a) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t j = blockIdx.y;
    const bool live = c < a.C;
    const int n = (int)a.n;
    const size_t stride = (size_t)a.d * (size_t)a.C;
    const double* col = a.s + (size_t)j * (size_t)a.C + (size_t)(live ? c : 0);
    double z[N];
#pragma unroll
    for (int t = 0; t < N; ++t) {
        if (t < N - 32) {
            z[t] = col[(size_t)t * stride];
        } else {                                               // the last 32 positions: rows past n read row n-1
            const double v = col[(size_t)(t < n ? t : n - 1) * stride];
            z[t] = t < n ? v : 0.0;
        }
    }
    const double nd = (double)n;
    // s / n for the autocovariances: q0 = RN(s rn), then one correction with the exact residual (fma).  With rn the
    // correctly rounded 1/n and q0 faithful, q0 + (s - n q0) rn rounds to the correctly rounded s / n (Markstein's
    // theorem; no underflow here): the IEEE quotient orc_ess computes, for 3 operations instead of the ~11 of a
    // division (tests/test_oracle.py checks the identity on half a billion quotients, near-exact ones included).
    const double rn = 1.0 / nd;
    auto qdiv = [&](double x) {
        const double q0 = x * rn;
        return __builtin_fma(__builtin_fma(-q0, nd, x), rn, q0);
    };
    double sum = 0.0;
#pragma unroll
    for (int t = 0; t < N; ++t) sum = sum + z[t];              // mean.jl:6, left to right; the zero pad adds +0
    const double mean = sum / nd;
#pragma unroll
    for (int t = 0; t < N; ++t) z[t] = (t < N - 32 || t < n) ? z[t] - mean : 0.0;
    // the lag-0 sum is ss (the same fma chain): it runs as the first of step 0's four chains
    double ss = 0.0, acv0 = 0.0;
    const int64_t k = (a.maxlag - 1) >= 0 ? (a.maxlag - 1) / 2 : -1;
    double gsum = 0.0, prev = 0.0;
    bool done = k < 0 || !live;
#pragma unroll
    for (int jp = 0; jp < N / 2; jp += 2) {                    // pairs jp, jp + 1: lags 2 jp .. 2 jp + 3
        if (jp > 0 && __ballot(!done) == 0) break;
        double sl[4] = {0.0, 0.0, 0.0, 0.0};
        auto lag_terms = [&](int t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int L = 2 * jp + i;
                if (t + L < N) sl[i] = __builtin_fma(z[t], z[t + L], sl[i]);
            }
        };
        // t in blocks of 4; once z[t + 2 jp] can be the zero pad (t + 2 jp >= N - 32), a block starting at or past
        // n - 2 jp (a uniform test) ends the sums: every term left is fma(z, 0, s) = s
#pragma unroll
        for (int tb = 0; tb < N; tb += 4) {
            if (tb + 2 * jp >= N - 32 && tb + 2 * jp >= n) break;
#pragma unroll
            for (int t = tb; t < tb + 4; ++t) lag_terms(t);
        }
        if (jp == 0) {
            ss = sl[0];
            acv0 = qdiv(ss);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int jj = jp + h;
            if (jj >= N / 2) break;
            const double g = (jj == 0 ? acv0 : qdiv(sl[2 * h])) + qdiv(sl[2 * h + 1]);   // acv[2j] + acv[2j+1]
            if (!done) done = jj > k || !geyer_take(g, jj, a.vtype, prev, gsum);
        }
    }
    if (live) {
        const double var_v = (-acv0 + 2.0 * gsum) / nd;
        const double var_iid = (ss / (nd - 1.0)) / nd;
        const size_t o = (size_t)j * (size_t)a.C + (size_t)c;
        a.ess[o] = (nd * var_iid) / var_v;                      // ess.jl:9
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
    if (vtype != 3 && n <= 96) {
        const dim3 grid((unsigned)((C + 255) / 256), (unsigned)d);
        if (n <= 32) k_ess_reg<32><<<grid, 256, 0, st>>>(a);
        else if (n <= 64) k_ess_reg<64><<<grid, 256, 0, st>>>(a);
        else k_ess_reg<96><<<grid, 256, 0, st>>>(a);
    } else if (n <= kEssTileMaxN) {
        const size_t lds = (size_t)kEssTile * ess_stride((int)n) * sizeof(double);
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
