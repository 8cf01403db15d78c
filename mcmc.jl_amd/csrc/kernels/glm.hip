// glm.hip -- regression models on fp64 MFMA: logistic (examples/logistic_regression.jl:16-22)
// and linear (examples/linear_regression.jl:14-20) log-targets with their gradients, fused into
// the RWM / MALA / HMC / HMCDA step loops.
//
// Mapping.  A wave owns a tile of 16 chains; the dense contractions are
//     eta[obs][chain] = X[obs][:] . beta[:][chain]        (v_mfma_f64_16x16x4_f64, K = coordinates)
//     G[coord][chain] = X[:][coord] . r[:][chain]          (same instruction, K = observations)
// per 16-observation tile of X staged in LDS and shared by the workgroup's waves.  Lane l holds
// chain cl = l & 15 and quarter q = l >> 4; for d-slice s (d > 64 is split over NW = d_pad/64
// waves) it owns coordinates k = s*DS + 16m + 4q + e (m < DS/16, e < 4), which are exactly the four
// normals of Philox blocks k/4 -- so proposals, momenta, gradients and every per-coordinate term
// stay lane-local.  The MFMA row <-> coordinate maps are permuted to make that so:
//     eta k-slice kk (= 4m + e), row q      <-> coordinate 16m + 4q + e
//     G tile T, row i (= 4r + q')           <-> coordinate 16T + 4q' + r
// and the eta accumulator (obs q + 4r on lane (q, cl)) is, register for register, the B operand
// of the G product (k-slice r): no data movement between the two MFMA chains.
//
// Arithmetic (restated by oracle/oracle.c orc_glm_eval): v_mfma_f64_16x16x4_f64 is a
// sequential fma chain over its k (probed bitwise on gfx950, scripts/probe_mfma.py), so eta is an
// fma chain over coordinates in (m, e, q) order per slice, slices added left to right; G is an fma
// chain over observations; per-coordinate sums are lane partials in (m, e) order combined as
// (q0 + q2) + (q1 + q3), then slices left to right.
#include <cstdlib>

#include "../common.hpp"
#include "../detmath.hpp"
#include "../models.hpp"
#include "../glm_layout.hpp"
#include "../ram.hpp"
#include "../host/kernels_api.hpp"

namespace mcmc {

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// workgroup: one slice (NW = 1): 4 waves = 4 tiles of 16 chains; d-sliced (NW = 2, 4, 8): 8 waves = 8 / NW tiles
template <int NW>
constexpr int glm_block() { return NW == 1 ? 256 : 512; }
constexpr int kGlmMaxWaves = 8;
#ifdef GLM_STAMP
constexpr int kGlmStampLdsBytes = 8 * 16 * 8 * 4;     // GLM_STAMP builds: the phase stamps' LDS (glm_eval)
#endif
// glm_eval1's elementwise schedule (the same operations either way): each sub-stage between
// eta MFMAs runs one stage of one observation row (0) or of all four rows of the lane (1)
#ifndef GLM_GROUP_ROWS
#define GLM_GROUP_ROWS 1
#endif
constexpr bool kGlmGroupRows = GLM_GROUP_ROWS != 0;
// 1: a scheduling fence after every elementwise sub-stage pins the eta MFMAs between them; 0 (default) leaves
// the interleaving to the compiler: config 3 runs 3.7 % faster without the fences
#ifndef GLM_FENCE
#define GLM_FENCE 0
#endif
constexpr bool kGlmFence = GLM_FENCE != 0;
// 1 (default): a fence after each k-slice of the G = X^T r MFMAs (operands one k-slice ahead)
#ifndef GLM_GFENCE
#define GLM_GFENCE 1
#endif
constexpr bool kGlmGFence = GLM_GFENCE != 0;
// 1 (default): single-slice MALA runs the wave-specialised glm_mala1ws (M and V waves paired on each SIMD);
// 0: glm_mala1 (one wave per tile does both)
#ifndef GLM_MALA1_WS
#define GLM_MALA1_WS 1
#endif
// glm_mala1ws: eta A operands read this many MFMAs ahead
#ifndef GLM_WS_LA
#define GLM_WS_LA 4
#endif
// GLM_WS_DMA (default 1): glm_mala1ws's V waves stage the X ring's tile t+2 by LDS-DMA (global_load_lds, no
// registers, no ds_write) instead of through registers
#ifndef GLM_WS_DMA
#define GLM_WS_DMA 1
#endif
// NM (template parameter) = DS/16 in {1, 2, 4, 8}: the lane owns NS = 4*NM coordinates.

struct GlmShape {
    int nw;          // waves per 16-chain tile (d-slices)
    int tpw;         // tiles per workgroup = max(4, nw) / nw
    int ds;          // coordinates per wave
    int nm;          // ds / 16
    int d_pad;
    int lds_stride;  // X tile row stride (doubles), glm_row_stride(d_pad)
    int ts;          // doubles per staged tile (rows, then Y), glm_tile_doubles(d_pad)
    int64_t n_pad;
};

struct GlmArgs {
    StepArgs s;
    SamplerArgs sa;
    ModelArgs m;
    ChainState st;
    GlmShape g;
    LeapRec rec;      // storeLeaps record (glm_hmc<..., REC = true>); zero otherwise
};

// lane position inside the workgroup
struct GlmPos {
    int lane, q, cl, wave, slice, tile;
    int64_t c;
    bool live;
    int base;
};

__device__ __forceinline__ GlmPos glm_pos(const GlmArgs& a) {
    GlmPos p;
    p.lane = threadIdx.x & 63;
    p.q = p.lane >> 4;
    p.cl = p.lane & 15;
    p.wave = threadIdx.x >> 6;
    p.slice = p.wave % a.g.nw;
    p.tile = p.wave / a.g.nw;
    const int64_t slot = ((int64_t)blockIdx.x * a.g.tpw + p.tile) * 16 + p.cl;
    p.live = slot < a.s.C;
    // every chain-indexed access below goes through p.c; a tile's MFMA columns are independent chains, so the
    // permutation changes which chains share a tile (and its leapfrog loop), never a chain's arithmetic
    p.c = (a.s.order != nullptr && p.live) ? (int64_t)a.s.order[slot] : slot;
    p.base = p.slice * a.g.ds;
    return p;
}

__device__ __forceinline__ int own_coord(const GlmPos& p, int slot) {
    return p.base + 16 * (slot >> 2) + 4 * p.q + (slot & 3);
}

// tile buffers in LDS (each glm_tile_doubles: 16 X rows in the glm_layout.hpp image, then Y): the d-sliced
// evaluation double-buffers, the single-slice one (glm_eval1) keeps three (tile t for G, t+1 for eta, t+2 being
// written); at d_pad = 1024 one tile is 129 KB, so the d-sliced evaluation keeps one (glm_eval: staged after the
// tile's last reader, behind a barrier)
__host__ __device__ constexpr int glm_xbufs(int nw, int d_pad) { return nw == 1 ? 3 : (d_pad > 512 ? 1 : 2); }

// LDS carve-up (doubles): tiles [xbufs][ts] | eta partials [8 waves][64][4] (single-slice kernels: the logistic
// term's table, kSoftplusTab, instead) | chain scalars [8 waves][16] | residual weights [4 tiles][4][64] | int scratch
struct GlmLds {
    double* X;
    double* part;
    double* scal;
    double* rbuf;     // [4 tiles][4 r][64 lanes]: residual weights of a tile, exchanged between slice waves
    int* iscr;
    double* beta;     // single-slice kernels: [4 waves][4 NM slots][64 lanes], a lane's proposal coordinates
};

__host__ __device__ constexpr int glm_part_doubles(int nw) {
    return nw == 1 && SP_NROWS * 10 > kGlmMaxWaves * 64 * 4 ? SP_NROWS * 10 : kGlmMaxWaves * 64 * 4;
}

__device__ __forceinline__ GlmLds glm_lds(const GlmArgs& a, double* smem) {
    GlmLds L;
    L.X = smem;
    L.part = L.X + glm_xbufs(a.g.nw, a.g.d_pad) * a.g.ts;                 // tile buffers
    L.scal = L.part + glm_part_doubles(a.g.nw);
    L.rbuf = L.scal + kGlmMaxWaves * 16;
    L.iscr = (int*)(L.rbuf + 4 * 4 * 64);
    L.beta = L.rbuf + 4 * 4 * 64 + 2;                // after the 4 ints of iscr
    return L;
}

static size_t glm_lds_bytes(const GlmShape& g) {
    return (size_t)(glm_xbufs(g.nw, g.d_pad) * g.ts + glm_part_doubles(g.nw) + kGlmMaxWaves * 16 +
                    4 * 4 * 64 + 2 + (g.nw == 1 ? 4 * 4 * g.nm * 64 : 0)) * 8
#ifdef GLM_STAMP
           + 16 + (g.nw > 1 ? kGlmStampLdsBytes : 0)
#endif
        ;
}

// sum of a per-chain quantity held as 4 quarter partials per wave and NW slice partials:
// (q0 + q2) + (q1 + q3), then slices left to right.  Contains a barrier when nw > 1:
// every wave of the workgroup must reach it.
__device__ __forceinline__ double glm_sum(const GlmArgs& a, const GlmPos& p, const GlmLds& L, double v) {
    v = v + __shfl_xor(v, 32, 64);
    v = v + __shfl_xor(v, 16, 64);
    if (a.g.nw == 1) return v;
    __syncthreads();
    if (p.q == 0) L.scal[p.wave * 16 + p.cl] = v;
    __syncthreads();
    double t = L.scal[(p.tile * a.g.nw) * 16 + p.cl];
    for (int s = 1; s < a.g.nw; ++s) t = t + L.scal[(p.tile * a.g.nw + s) * 16 + p.cl];
    return t;
}

// workgroup-wide max of a per-chain integer (leapfrog counts): every wave must reach it.
__device__ __forceinline__ int64_t glm_max(const GlmLds& L, int64_t v, bool live) {
    __syncthreads();
    if (threadIdx.x == 0) L.iscr[0] = 1;
    __syncthreads();
    if (live) atomicMax(&L.iscr[0], (int)v);
    __syncthreads();
    const int r = L.iscr[0];
    __syncthreads();
    return r;
}

// the workgroup-wide max of a per-chain integer and the max over this wave's chain tile (d-sliced geometry: at most
// two tiles a workgroup); every wave must reach it
__device__ __forceinline__ int64_t glm_max_tile(const GlmLds& L, int64_t v, bool live, int tile, int64_t& tmax) {
    __syncthreads();
    if (threadIdx.x == 0) {
        L.iscr[0] = 1;
        L.iscr[1] = 1;
        L.iscr[2] = 1;
    }
    __syncthreads();
    if (live) {
        atomicMax(&L.iscr[0], (int)v);
        atomicMax(&L.iscr[1 + tile], (int)v);
    }
    __syncthreads();
    const int r = L.iscr[0];
    tmax = L.iscr[1 + tile];
    __syncthreads();
    return r;
}

// The lane's coordinates of the evaluation point: held in registers (XArr) or in the lane's private
// LDS slots (XLds: slot s at b[64 s], b = L.beta + (wave * 4 NM) * 64 + lane).
template <int NS>
struct XArr {
    const double (&v)[NS];
    __device__ __forceinline__ double operator()(int s) const { return v[s]; }
};
struct XLds {
    const double* b;
    __device__ __forceinline__ double operator()(int s) const { return b[64 * s]; }
};

// The end of an evaluation: likelihood partials combined (quarters, then slices left to right), the
// prior vars ~ Normal(0, sp) over own coordinates, the LLAcc rule, and the prior's gradient added to G.
template <int NM, int NW, bool GRAD, class XA>
__device__ __forceinline__ double glm_finish(const GlmArgs& a, const GlmPos& p, const GlmLds& L,
                                          const XA& x, f64x4 (&G)[NM], double lik_part, bool& oos, bool on = true) {
    const ModelArgs& M = a.m;
    const int d = M.d;
    const double lik = glm_sum(a, p, L, lik_part);
    // prior vars ~ Normal(0, sp) over own coordinates
    const double sp = M.prior_sigma, s2p = sp * sp, logsp = det_log(sp);
    double pp = 0.0;
#pragma unroll
    for (int slot = 0; slot < (4 * NM); ++slot) {
        const int k = own_coord(p, slot);
        if (true && k < d) {
            const double z = (x(slot) - 0.0) / sp;
            pp = pp + (-0.5 * (z * z + kLog2Pi) - logsp);
        }
    }
    const double prior = glm_sum(a, p, L, pp);
    double acc = 0.0 + prior;                                           // LLAcc(0.) + ...
    bool bad = !(acc - acc == 0.0);
    acc = acc + lik;
    bad = bad || !(acc - acc == 0.0);
    oos = bad;
    if (bad) acc = -__builtin_inf();
    if (GRAD && on) {
#pragma unroll
        for (int slot = 0; slot < (4 * NM); ++slot)
            G[slot >> 2][slot & 3] = bad ? 0.0 : (0.0 - x(slot)) / s2p + G[slot >> 2][slot & 3];
    }
    return acc;
}

// The probit model's elementwise part for one observation (examples/probit_regression.jl:26-40; oracle orc_glm_eval):
// term = y logcdf(N, eta) + (1 - y) logcdf(N, -eta), and its eta-derivative, the example's grad_log_posterior weight
// y exp(A - logcdf(N, eta)) - (1 - y) exp(A - logcdf(N, -eta)), A = -(eta^2 + log(2 pi))/2
__device__ __forceinline__ void glm_probit_obs(double eta, double y, double& term, double& w) {
    const double la = det_normlogcdf(eta), lb = det_normlogcdf(-eta);
    term = y * la + (1.0 - y) * lb;
    const double A = (-(eta * eta + kLog2Pi)) / 2.0;
    w = y * det_exp(A - la) - (1.0 - y) * det_exp(A - lb);
}

// Single-slice evaluation (NW = 1: the wave holds all d_pad coordinates of its 16 chains), software
// pipelined over the 16-observation tiles with three LDS tile buffers:
//     iteration t:  eta_{t+1} = X_{t+1} beta   (MFMA chain, buffer (t+1) % 3)
//                   elementwise on eta_t        (VALU, independent of the chain above: the two interleave)
//                   G += X_t^T r_t              (MFMA, buffer t % 3)
//                   tile t+2 -> buffer (t+2) % 3 (its last readers finished before the previous barrier)
//                   one barrier
// The arithmetic is glm_eval's, operation for operation (eta chains over (m, e, q); G chains over
// observations; a lane's likelihood terms in (t, r) order), so the oracle's orc_glm_eval restates both.
template <int NM, bool GRAD, bool LOGI, class XA>
__device__ __forceinline__ double glm_eval1_tiles(const GlmArgs& a, const GlmPos& p, const GlmLds& L,
                                                const XA& x, f64x4 (&G)[NM]) {
    const ModelArgs& M = a.m;
    const GlmShape& g = a.g;
    constexpr int S = glm_row_stride(16 * NM);
    const bool probit = !LOGI && M.kind == MK_PROBIT;          // probit runs in the linear instantiation (uniform)
    const double sn = M.noise_sigma, s2n = sn * sn;
    const double logsn = LOGI ? 0.0 : det_log(sn);
    const double isn = 1.0 / sn, is2n = 1.0 / s2n;
    double lik_part = 0.0;
    const int64_t ntiles = g.n_pad / 16;
    constexpr int kBlk = glm_block<1>();
    constexpr int DP = 16 * NM;
    constexpr int XS = glm_tile_doubles(DP);                  // one staged tile: X rows, then Y
    constexpr int YO = glm_y_offset(DP);
    constexpr int BO = glm_b_offset(DP);
    constexpr int kHalf = XS / 2;                             // f64x2 per tile
    constexpr int kPer = (kHalf + kBlk - 1) / kBlk;
    static_assert(glm_row_stride(DP) > 0, "");
    f64x2 buf[kPer];
    // the tile image moves linearly (glm_layout.hpp): HBM tile tt -> LDS buffer b
    auto load_tile = [&](int64_t tt) {
        const f64x2* src = reinterpret_cast<const f64x2*>(M.X + (size_t)tt * XS);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int i = threadIdx.x + kBlk * j;
            buf[j] = src[i < kHalf ? i : 0];
        }
    };
    auto store_tile = [&](int b) {
        f64x2* dst = reinterpret_cast<f64x2*>(L.X + b * XS);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int i = threadIdx.x + kBlk * j;
            if (i < kHalf) dst[i] = buf[j];
        }
    };
    const int eta_lane = p.cl * S + 4 * p.q;              // + glm_eta_off(slot): coordinate 16m + 4q + e
    // eta of the tile in buffer b: k-slice kk = 4m + e, row q <-> coordinate 16m + 4q + e
    auto eta_of = [&](int b) {
        f64x4 e = f64x4{0.0, 0.0, 0.0, 0.0};
        const double* xrow = L.X + b * XS + eta_lane;
#pragma unroll
        for (int slot = 0; slot < (4 * NM); ++slot)
            e = __builtin_amdgcn_mfma_f64_16x16x4f64(xrow[glm_eta_off(slot)], x(slot), e, 0, 0, 0);
        return e;
    };
    load_tile(0);
    store_tile(0);
    if (ntiles > 1) {
        load_tile(1);
        store_tile(1);
    }
    // logistic: the term's segment-polynomial table (det_logi) staged in the eta-partials area, which the
    // single-slice kernels do not otherwise use
    const double (*sptab)[10] = reinterpret_cast<const double (*)[10]>(L.part);
    if (LOGI) {
        for (int i = threadIdx.x; i < SP_NROWS * 10; i += kBlk) L.part[i] = (&kSoftplusTab[0][0])[i];
    }
    if (GRAD) {
#pragma unroll
        for (int T = 0; T < NM; ++T) G[T] = f64x4{0.0, 0.0, 0.0, 0.0};
    }
    __syncthreads();
    f64x4 eta = eta_of(0);
    double ubnd = -__builtin_inf();                           // logistic: max of u + b over the lane's observations
    const int64_t nfull = M.n / 16;                           // tiles without padded observations
    int b = 0;                                                // buffer of tile t
    for (int64_t t = 0; t < ntiles; ++t) {
        const bool more = t + 2 < ntiles;
        if (more) load_tile(t + 2);
        const int b1 = b == 2 ? 0 : b + 1, b2 = b1 == 2 ? 0 : b1 + 1;
        // eta_{t+1} (buffer b1; garbage past the last tile, unused) interleaved with the elementwise work on
        // eta_t by hand: the four rows' work runs in stages (det_exp / det_log split at their natural points,
        // the same operations), 32 sub-stages (stage, row) per tile, and sub-stage j is preceded by the
        // eta MFMAs [j KM / 32, (j+1) KM / 32), KM = 4 NM; a scheduling fence after every sub-stage keeps that
        // order (an in-order wave can only overlap a dependent MFMA chain with VALU placed between its MFMAs).
        // The eta operands are read from LDS kLA MFMAs ahead.
        constexpr int KM = 4 * NM;
        constexpr int kLA = 4;
        f64x4 eta_next = f64x4{0.0, 0.0, 0.0, 0.0};
        const double* xrow1 = L.X + b1 * XS + eta_lane;
        const double* LY = L.X + b * XS + YO;
        const double* LB = L.X + b * XS + BO;
        double av[KM];
#pragma unroll
        for (int m = 0; m < (kLA < KM ? kLA : KM); ++m) av[m] = xrow1[glm_eta_off(m)];
        double y[4], bnd[4], term[4], rv[4];                    // y: the response, for the logistic model w (det_logi)
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = LY[p.q + 4 * r];
        if (LOGI) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bnd[r] = LB[p.q + 4 * r];
        }
        // sub-stage j: the eta MFMAs [j KM / NSUB, (j+1) KM / NSUB), then stage st of one row (kGlmGroupRows
        // false) or of all four rows, four independent dependency chains (kGlmGroupRows true)
        // logistic: one row's whole det_logi a sub-stage (its state stays in registers only that long)
        constexpr int NSTAGE = 1;
        constexpr bool GR = LOGI ? false : kGlmGroupRows;
        constexpr int NSUB = GR ? NSTAGE : 4 * NSTAGE;
#pragma unroll
        for (int j = 0; j < NSUB; ++j) {
#pragma unroll
            for (int m = j * KM / NSUB; m < (j + 1) * KM / NSUB; ++m) {
                if (m + kLA < KM) av[m + kLA] = xrow1[glm_eta_off(m + kLA)];
                eta_next = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m], x(m), eta_next, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (!GR && r != (j & 3)) continue;
                if (LOGI) {
                    // prob = 1/(1+exp(-X*vars)); Y ~ Bernoulli(prob); its eta-derivative (MCMCDerivRules.jl:111)
                    LogiState E;
                    det_logi_s1(eta[r], y[r], E, sptab);
                    ubnd = __builtin_fmax(ubnd, E.u + bnd[r]);                    // the reference's -Inf
                    det_logi_s2(E);
                    det_logi_fin(E, y[r], term[r], rv[r]);
                } else if (probit) {
                    glm_probit_obs(eta[r], y[r], term[r], rv[r]);
                } else {
                    const double resid = y[r] - eta[r];                             // resid = Y - X*vars
                    const double z = resid * isn;
                    term[r] = -0.5 * (z * z + kLog2Pi) - logsn;                     // resid ~ Normal(0, sn)
                    rv[r] = resid * is2n;
                }
            }
            if (kGlmFence) __builtin_amdgcn_sched_barrier(0);
        }
        if (t < nfull) {                                                        // uniform: no padded observation
#pragma unroll
            for (int r = 0; r < 4; ++r) lik_part = lik_part + term[r];          // the lane's terms in (t, r) order
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool in = t * 16 + p.q + 4 * r < M.n;
                lik_part = in ? lik_part + term[r] : lik_part;
                rv[r] = in ? rv[r] : 0.0;
            }
        }
        if (GRAD) {
            // G tile T, k-slice kk: A[i][k] = X[obs 4kk+q][coord 16T+4(i&3)+(i>>2)], i = cl; kk outer so that
            // consecutive MFMAs feed independent accumulators; operands one kk ahead
            const double* gcol = L.X + b * XS + p.q * S + 4 * (p.cl & 3) + (p.cl >> 2);
            double ga[NM];
#pragma unroll
            for (int T = 0; T < NM; ++T) ga[T] = gcol[glm_g_off(T)];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                double gn[NM];
                if (kk < 3) {
#pragma unroll
                    for (int T = 0; T < NM; ++T) gn[T] = gcol[4 * (kk + 1) * S + glm_g_off(T)];
                }
#pragma unroll
                for (int T = 0; T < NM; ++T) G[T] = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[T], rv[kk], G[T], 0, 0, 0);
                if (kGlmGFence) __builtin_amdgcn_sched_barrier(0);
                if (kk < 3) {
#pragma unroll
                    for (int T = 0; T < NM; ++T) ga[T] = gn[T];
                }
            }
        }
        if (more) store_tile(b2);                             // held tile t-1: read before the last barrier
        __syncthreads();
        eta = eta_next;
        b = b1;
    }
    return LOGI && ubnd >= 0.0 ? -__builtin_inf() : lik_part;
}

template <int NM, bool GRAD, class XA>
__device__ __forceinline__ double glm_eval1(const GlmArgs& a, const GlmPos& p, const GlmLds& L,
                                         const XA& x, f64x4 (&G)[NM], bool& oos) {
    const double lik_part = a.m.kind == MK_LOGISTIC ? glm_eval1_tiles<NM, GRAD, true>(a, p, L, x, G)
                                                    : glm_eval1_tiles<NM, GRAD, false>(a, p, L, x, G);
    return glm_finish<NM, 1, GRAD>(a, p, L, x, G, lik_part, oos);
}

// LDS-DMA of staged tile tt into an LDS buffer: the image is contiguous (glm_layout.hpp), so each wave moves whole
// 1-KiB pieces (global_load_lds_dwordx4: LDS M0 + 16 lane bytes), pieces w, w + 8, ... of the tile.  The copy is
// counted on vmcnt only: the reader waits vmcnt(0) (glm_dma_wait) and passes a barrier after it (glm_eval).
// Written as inline asm: the compiler's waitcnt pass treats a __builtin_amdgcn_global_load_lds as an LDS store
// that may alias every later ds_write, and put an s_waitcnt vmcnt(0) before the eta-partial store right after the
// eta MFMAs -- draining the next tile's copy a few hundred cycles after it was issued (r04 ISA).  The asm is
// opaque to that pass.  The LDS address goes in through the "{m0}" operand constraint: the compiler writes M0
// itself and knows what it holds afterwards (M0 is a reserved register, so a clobber would not be honoured).
// Loads the pass does track stay correctly waited for: vmcnt decrements in issue order, so an extra load in flight
// only makes its counted waits longer.
template <int TS>
constexpr int glm_dma_pieces_per_wave() { return (TS / 128 + 7) / 8; }
// piece j (0 <= j < glm_dma_pieces_per_wave) of this wave's share of tile image img -> LDS buffer buf
template <int TS>
__device__ __forceinline__ void glm_dma_piece(const double* img, double* buf, int j) {
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    constexpr int kPieces = TS / 128;
    const int c = w + 8 * j;
    if (c < kPieces) {
        const double* src = img + c * 128 + 2 * lane;
        const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(uintptr_t)buf + (uint32_t)c * 1024u));
        asm volatile("global_load_lds_dwordx4 %0, off" :: "v"(src), "{m0}"(lds) : "memory");
    }
}
template <int TS>
__device__ __forceinline__ void glm_dma_tile(const double* img, double* buf) {
#pragma unroll
    for (int j = 0; j < glm_dma_pieces_per_wave<TS>(); ++j) glm_dma_piece<TS>(img, buf, j);
}
// tile image img -> LDS buffer buf by the NWV waves of one role (w: the wave's index among them, wave-uniform),
// pieces w, w + NWV, ... (glm_mala1ws: the V waves stage the X ring)
template <int TS, int NWV>
__device__ __forceinline__ void glm_dma_tile_w(const double* img, double* buf, int w) {
    constexpr int kPieces = TS / 128;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < (kPieces + NWV - 1) / NWV; ++j) {
        const int c = w + NWV * j;
        if (c < kPieces) {
            const double* src = img + c * 128 + 2 * lane;
            const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(uintptr_t)buf + (uint32_t)c * 1024u));
            asm volatile("global_load_lds_dwordx4 %0, off" :: "v"(src), "{m0}"(lds) : "memory");
        }
    }
}
// GLM_DMA_SPREAD (default 2; 0: off): the next tile's pieces issued between the eta MFMAs, one after every
// GLM_DMA_SPREAD-th MFMA, instead of all before the eta operand reads (round 6, config 5: 0.584 -> 0.605 of the fp64
// spec, profiles/r06_ab_glm.md)
// GLM_ETA_LA (default 8): how many eta A-operand reads run ahead of their MFMA in the 128-wide slices (NM = 8; the
// 64-wide slices read all 16 before the first MFMA)
#ifndef GLM_ETA_LA
#define GLM_ETA_LA 8
#endif
#ifndef GLM_DMA_SPREAD
#define GLM_DMA_SPREAD 2
#endif
// GLM_TILE_SKIP (default 1): in glm_hmc's d-sliced trajectories a chain tile whose chains have all finished skips
// its evaluations' MFMA and elementwise work for the rest of the workgroup's trajectory
#ifndef GLM_TILE_SKIP
#define GLM_TILE_SKIP 1
#endif
// a workgroup barrier for LDS data written by ds_write (lgkmcnt) that leaves LDS-DMAs in flight: __syncthreads()
// would also wait vmcnt(0), draining the next tile's copy (cdna_hip_programming.md §5, pipelining across barriers)
__device__ __forceinline__ void glm_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void glm_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// GLM_STAMP (dev build only, scripts/glm_stamps.py): shader-clock stamps (low 32 bits) of the d-sliced tile loop's
// phases, every wave of workgroups 0..3, tiles 8..23 of the last evaluation (the points: loop top, eta partial
// stored, barrier 1, weights stored, barrier 2, G issued, tile t+1 landed, barrier 3).  They are kept in 4 KB of LDS
// past the kernel's own (global stores inside the loop would count on vmcnt and stretch the DMA wait they measure)
// and copied out after the loop.
#ifdef GLM_STAMP
static __device__ unsigned g_glm_stamps[4][8][16][8];
#define GLM_STAMPT(pt)                                                                                  \
    do {                                                                                               \
        if (t >= 8 && t < 24) {                                                                        \
            const unsigned ts_ = (unsigned)__builtin_amdgcn_s_memtime();                              \
            if ((threadIdx.x & 63) == 0) stamp_lds[((threadIdx.x >> 6) * 16 + (t - 8)) * 8 + (pt)] = ts_; \
        }                                                                                              \
    } while (0)
#else
#define GLM_STAMPT(pt) do { } while (0)
#endif

// log-target and (GRAD) gradient of the regression model at the lane's coordinates x.
// Every wave of the workgroup calls it the same number of times (barriers inside).
// gout doubles as the MFMA accumulator of G = X^T r (G[T] covers slots 4T..4T+3).
//
// d-sliced form (NW = 2, 4, 8 slices of DS = 16 NM = 128 coordinates; 8 / NW tiles of 16 chains per workgroup):
// per 16-observation tile t, in LDS buffer t & 1 (one buffer at d_pad = 1024),
//     LDS-DMA of tile t+1 into the other buffer (issued first, waited for at the end of the iteration)
//     eta partial over the wave's slice (NM k-groups of MFMAs, operands read kLA ahead)  -> part[wave]
//     barrier; the slice wave owning row r of its tile adds the NW partials left to right, the likelihood term and
//     residual weight of that row -> rbuf[tile][r]
//     barrier; every wave reads its tile's 4 rows' weights; G += X_t^T r (NM independent accumulators)
//     vmcnt(0) + barrier: tile t+1 has landed and tile t's buffer, part and rbuf are free again.
// Two tiles of chains share each staged tile (reuse 32 chains per X byte from L2 / MALL).
// on = false (wave-uniform; a chain tile whose every chain has finished its trajectory, glm_hmc): the wave takes its
// share of the staging and every barrier, and skips its MFMAs and elementwise work; G is left as it is and the
// returned value is not the log-target (the caller keeps its own).
template <int NM, int NW, bool GRAD>
__device__ __forceinline__ double glm_eval(const GlmArgs& a, const GlmPos& p, const GlmLds& L,
                                        const double (&x)[(4 * NM)], f64x4 (&G)[NM], bool& oos, bool on = true) {
    if constexpr (NW == 1) return glm_eval1<NM, GRAD>(a, p, L, XArr<4 * NM>{x}, G, oos);
    const ModelArgs& M = a.m;
    const GlmShape& g = a.g;
    constexpr int DP = 16 * NM * NW;
    constexpr int S = glm_row_stride(DP);
    constexpr int XS = glm_tile_doubles(DP);
    constexpr int YO = glm_y_offset(DP);
    constexpr int BO = glm_b_offset(DP);
    constexpr bool kOneBuf = DP > 512;                        // glm_xbufs: one LDS tile buffer
    const bool logistic = M.kind == MK_LOGISTIC;
    const double sn = M.noise_sigma, s2n = sn * sn;
    const double logsn = logistic ? 0.0 : det_log(sn);
    const double isn = 1.0 / sn, is2n = 1.0 / s2n;
    if (GRAD && on) {
#pragma unroll
        for (int T = 0; T < NM; ++T) G[T] = f64x4{0.0, 0.0, 0.0, 0.0};
    }
    double lik_part = 0.0;
    double ubnd = -__builtin_inf();                           // logistic: max of u + b over the lane's observations
    const int64_t ntiles = g.n_pad / 16;
    const int eta_lane = p.cl * S + 4 * p.q + p.base;                       // + glm_eta_off(slot)
    const int g_lane = p.q * S + 4 * (p.cl & 3) + (p.cl >> 2) + p.base;   // + 4 kk S + glm_g_off(T)
#ifdef GLM_STAMP
    unsigned* const stamp_lds = reinterpret_cast<unsigned*>(L.iscr + 4);
#endif
    glm_dma_tile<XS>(M.X, L.X);
    glm_dma_wait();
    __syncthreads();
    for (int64_t t = 0; t < ntiles; ++t) {
        GLM_STAMPT(0);
        const int b = kOneBuf ? 0 : (int)(t & 1);
        const double* LX = L.X + b * XS;
        const bool more = t + 1 < ntiles;
        const double* const nimg = M.X + (size_t)(t + 1) * XS;
        double* const nbuf = L.X + (b ^ 1) * XS;
        // the wave's share of tile t+1's DMA: spread over its eta MFMAs (GLM_DMA_SPREAD), all here without them
        if ((!GLM_DMA_SPREAD || !on) && more && !kOneBuf) glm_dma_tile<XS>(nimg, nbuf);
        // eta partial over this wave's coordinates: k-slice kk = 4m + e, row q <-> coord base+16m+4q+e.  Every operand
        // read is issued before the first MFMA (a scheduling fence keeps them there: left alone, the scheduler sank
        // each read next to its MFMA and the chain waited out every LDS round trip); the waitcnt pass then waits
        // for each MFMA's own read only.
        constexpr int RPW = NW >= 4 ? 1 : 4 / NW;
        const int r0 = p.slice * RPW;
        const double* LY = LX + YO;
        double yv[RPW], bv[RPW];
#pragma unroll
        for (int rr_ = 0; rr_ < RPW; ++rr_) yv[rr_] = LY[p.q + 4 * ((r0 + rr_) & 3)];
        if (logistic) {
#pragma unroll
            for (int rr_ = 0; rr_ < RPW; ++rr_) bv[rr_] = LX[BO + p.q + 4 * ((r0 + rr_) & 3)];
        }
        f64x4 eta = f64x4{0.0, 0.0, 0.0, 0.0};
        if (on) {
            constexpr int KM = 4 * NM;
            constexpr int kLA = NM <= 4 ? KM : GLM_ETA_LA;
            const double* xrow = LX + eta_lane;
            double av[KM];
#pragma unroll
            for (int m = 0; m < kLA; ++m) av[m] = xrow[glm_eta_off(m)];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < KM; ++m) {
                if (m + kLA < KM) av[m + kLA] = xrow[glm_eta_off(m + kLA)];
                eta = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m], x[m], eta, 0, 0, 0);
                constexpr int SP = GLM_DMA_SPREAD > 0 ? GLM_DMA_SPREAD : 1;
                if (GLM_DMA_SPREAD && !kOneBuf && m % SP == SP - 1 && m / SP < glm_dma_pieces_per_wave<XS>()) {
                    if (more) glm_dma_piece<XS>(nimg, nbuf, m / SP);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (GLM_DMA_SPREAD && !kOneBuf && more) {
                constexpr int SP = GLM_DMA_SPREAD > 0 ? GLM_DMA_SPREAD : 1;
#pragma unroll
                for (int j = KM / SP; j < glm_dma_pieces_per_wave<XS>(); ++j) glm_dma_piece<XS>(nimg, nbuf, j);
            }
        }
        // Elementwise part, split over the slice waves: wave slice s owns observation rows r in
        // [s*RPW, (s+1)*RPW) of its tile (obs 16t + q + 4r for lane (q, cl)); with NW = 8 slices 4..7 own
        // none.  Its eta is the slices' partials added left to right.  Partials are [wave][r][lane] (lane-contiguous
        // 8-byte stores and loads: no bank conflicts), all NW of a row read before the first add.
        {
            double* mine = L.part + p.wave * 256 + p.lane;
#pragma unroll
            for (int r = 0; r < 4; ++r) mine[64 * r] = eta[r];
        }
        GLM_STAMPT(1);
        glm_lds_barrier();
        GLM_STAMPT(2);
        double rv[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int rr_ = 0; rr_ < RPW; ++rr_) {
            const int r = r0 + rr_;
            if (r >= 4 || !on) break;
            double pe[NW];
#pragma unroll
            for (int sl = 0; sl < NW; ++sl) pe[sl] = L.part[(p.tile * NW + sl) * 256 + r * 64 + p.lane];
            double e = pe[0];
#pragma unroll
            for (int sl = 1; sl < NW; ++sl) e = e + pe[sl];
            const int64_t obs = t * 16 + p.q + 4 * r;
            const double y = yv[rr_];
            double term, w;
            if (logistic) {
                // prob = 1/(1+exp(-X*vars)); Y ~ Bernoulli(prob); MCMCDerivRules.jl:111 (y: the image's w, det_logi)
                LogiState E;
                det_logi_s1(e, y, E);
                ubnd = __builtin_fmax(ubnd, E.u + bv[rr_]);                  // the reference's -Inf (logi_bound)
                det_logi_s2(E);
                det_logi_fin(E, y, term, w);
            } else if (M.kind == MK_PROBIT) {
                glm_probit_obs(e, y, term, w);
            } else {
                const double resid = y - e;                             // resid = Y - X*vars
                const double z = resid * isn;
                term = -0.5 * (z * z + kLog2Pi) - logsn;                // resid ~ Normal(0, sn)
                w = resid * is2n;
            }
            const bool in = obs < M.n;
            if (in) lik_part = lik_part + term;
            rv[rr_] = in ? w : 0.0;
        }
        // G tile T, k-slice kk': A[i][k] = X[obs 4kk'+q][coord base+16T+4(i&3)+(i>>2)], i = cl; kk outer so that
        // consecutive MFMAs feed independent accumulators.  NM <= 4: all 4 NM operands are read before the weights
        // barrier (they do not depend on it); NM = 8: one k-slice ahead.
        constexpr int kGA = NM <= 4 ? 4 : 1;                      // k-slices of operands read up front
        const double* gcol = LX + g_lane;
        double ga[4][NM];
        if (GRAD && on) {
#pragma unroll
            for (int kk = 0; kk < kGA; ++kk)
#pragma unroll
                for (int T = 0; T < NM; ++T) ga[kk][T] = gcol[4 * kk * S + glm_g_off(T)];
        }
        {
            // publish the owned rows' weights, then every slice wave reads all four for its G product
            double* rb = L.rbuf + p.tile * 256;
#pragma unroll
            for (int rr_ = 0; rr_ < RPW; ++rr_)
                if (r0 + rr_ < 4) rb[(r0 + rr_) * 64 + p.lane] = rv[rr_];
            GLM_STAMPT(3);
            glm_lds_barrier();
            GLM_STAMPT(4);
#pragma unroll
            for (int r = 0; r < 4; ++r) rv[r] = rb[r * 64 + p.lane];
        }
        if (GRAD && on) {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                if (kGA == 1 && kk < 3) {
#pragma unroll
                    for (int T = 0; T < NM; ++T) ga[kk + 1][T] = gcol[4 * (kk + 1) * S + glm_g_off(T)];
                }
#pragma unroll
                for (int T = 0; T < NM; ++T)
                    G[T] = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[kk][T], rv[kk], G[T], 0, 0, 0);
            }
        }
        if (kOneBuf) {                                        // the one buffer: after its last reader of tile t
            __syncthreads();
            if (more) glm_dma_tile<XS>(M.X + (size_t)(t + 1) * XS, L.X);
        }
        GLM_STAMPT(5);
        glm_dma_wait();                                       // tile t+1 landed (this wave's pieces) ...
        GLM_STAMPT(6);
        __syncthreads();                                      // ... and every wave's; buffers, part, rbuf free
        GLM_STAMPT(7);
    }
#ifdef GLM_STAMP
    if (blockIdx.x < 4 && (threadIdx.x & 63) == 0)
        for (int j = 0; j < 16 * 8; ++j) (&g_glm_stamps[blockIdx.x][threadIdx.x >> 6][0][0])[j] = stamp_lds[(threadIdx.x >> 6) * 128 + j];
#endif
    return glm_finish<NM, NW, GRAD>(a, p, L, XArr<4 * NM>{x}, G, logistic && ubnd >= 0.0 ? -__builtin_inf() : lik_part,
                                    oos, on);
}

// ------------------------------------------------------------------ state access (layout [d][ld])
// Lane pointer at coordinate base + 4q; slot (m, e) adds the wave-uniform offset (16m + e) * ld,
// so the 32 slot addresses cost SGPRs, not VGPRs.
// The pointer passes through an empty volatile asm at every use: the per-slot addresses derived from it are then
// formed where they are used instead of being hoisted out of the step / leapfrog loops, where 4 NM 64-bit addresses per
// state array stayed live across the tile loop and spilled (glm_hmc<8, 4> needed > 1.3 KB of scratch a lane).
template <class T>
__device__ __forceinline__ T* glm_lane_ptr(const GlmPos& p, T* base, int64_t ld, int64_t c) {
    T* r = base + (size_t)(p.base + 4 * p.q) * (size_t)ld + (size_t)c;
    asm volatile("" : "+v"(r));
    return r;
}
__device__ __forceinline__ bool glm_valid(const GlmArgs& a, const GlmPos& p, int slot) {
    return own_coord(p, slot) < a.s.d;
}
// an unconditional load's offset from the lane pointer (row base + 4q of the chain) to slot `slot`'s row, or, for a
// slot past d, to the chain's row 0: the state holds d rows, and the lane's own row base + 4q is past them too when
// d is not a multiple of the slice geometry (d = 300: rows 300..511; the loaded value is zeroed either way)
__device__ __forceinline__ ptrdiff_t glm_slot_off(const GlmArgs& a, const GlmPos& p, int slot, size_t ld) {
    return glm_valid(a, p, slot) ? (ptrdiff_t)(16 * (slot >> 2) + (slot & 3)) * (ptrdiff_t)ld
                                 : -(ptrdiff_t)(p.base + 4 * p.q) * (ptrdiff_t)ld;
}
template <int NM>
__device__ __forceinline__ void glm_load(const GlmArgs& a, const GlmPos& p, const double* src,
                                         double (&v)[(4 * NM)]) {
    const double* lp = glm_lane_ptr(p, src, a.s.ld, p.live ? p.c : 0);
    const size_t ld = (size_t)a.s.ld;
#pragma unroll
    for (int slot = 0; slot < (4 * NM); ++slot)
        v[slot] = glm_valid(a, p, slot) ? lp[(size_t)(16 * (slot >> 2) + (slot & 3)) * ld] : 0.0;
}
// glm_load with unconditional loads (an invalid slot reads the chain's row 0 and is zeroed): no masked load and wait
// per slot, every load in flight together -- for kernels that load the state once and have the registers for it
// (the evaluation kernel); in the step kernels the compiler then keeps the loads live across the step and spills
template <int NM>
__device__ __forceinline__ void glm_load_all(const GlmArgs& a, const GlmPos& p, const double* src,
                                             double (&v)[(4 * NM)]) {
    const double* lp = glm_lane_ptr(p, src, a.s.ld, p.live ? p.c : 0);
    const size_t ld = (size_t)a.s.ld;
#pragma unroll
    for (int slot = 0; slot < (4 * NM); ++slot) {
        const bool ok = glm_valid(a, p, slot);
        const double t = lp[glm_slot_off(a, p, slot, ld)];
        v[slot] = ok ? t : 0.0;
    }
}
template <int NM>
__device__ __forceinline__ void glm_store(const GlmArgs& a, const GlmPos& p, double* dst, int64_t ldd,
                                          const double (&v)[(4 * NM)]) {
    if (!p.live) return;
    double* lp = glm_lane_ptr(p, dst, ldd, p.c);
    const size_t ld = (size_t)ldd;
#pragma unroll
    for (int slot = 0; slot < (4 * NM); ++slot)
        if (glm_valid(a, p, slot)) lp[(size_t)(16 * (slot >> 2) + (slot & 3)) * ld] = v[slot];
}
template <int NM>
__device__ __forceinline__ void glm_store_kept(const GlmArgs& a, const GlmPos& p, int64_t kk, double* base,
                                               const double (&v)[(4 * NM)]) {
    if (base == nullptr) return;
    glm_store<NM>(a, p, base + (size_t)kk * (size_t)a.s.d * (size_t)a.s.C, a.s.C, v);
}
template <int NM>
__device__ __forceinline__ void glm_load4(const GlmArgs& a, const GlmPos& p, const double* src,
                                          f64x4 (&v)[NM]) {
    const double* lp = glm_lane_ptr(p, src, a.s.ld, p.live ? p.c : 0);
    const size_t ld = (size_t)a.s.ld;
#pragma unroll
    for (int slot = 0; slot < (4 * NM); ++slot)
        v[slot >> 2][slot & 3] = glm_valid(a, p, slot) ? lp[(size_t)(16 * (slot >> 2) + (slot & 3)) * ld] : 0.0;
}
template <int NM>
__device__ __forceinline__ void glm_store4(const GlmArgs& a, const GlmPos& p, double* dst, int64_t ldd,
                                           const f64x4 (&v)[NM]) {
    if (!p.live) return;
    double* lp = glm_lane_ptr(p, dst, ldd, p.c);
    const size_t ld = (size_t)ldd;
#pragma unroll
    for (int slot = 0; slot < (4 * NM); ++slot)
        if (glm_valid(a, p, slot)) lp[(size_t)(16 * (slot >> 2) + (slot & 3)) * ld] = v[slot >> 2][slot & 3];
}
template <int NM>
__device__ __forceinline__ void glm_store_kept4(const GlmArgs& a, const GlmPos& p, int64_t kk, double* base,
                                                const f64x4 (&v)[NM]) {
    if (base == nullptr) return;
    glm_store4<NM>(a, p, base + (size_t)kk * (size_t)a.s.d * (size_t)a.s.C, a.s.C, v);
}
// add the tile's evaluation counts to the launch-wide counter (one atomic per wave)
__device__ __forceinline__ void glm_count_evals(const GlmArgs& a, const GlmPos& p, int64_t n) {
    if (a.s.n_evals == nullptr) return;
    unsigned long long v = (p.live && p.q == 0 && p.slice == 0) ? (unsigned long long)n : 0ull;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if (p.lane == 0) atomicAdd(a.s.n_evals, v);
}
// the tile's accept bits of a kept step (called by every lane of the wave): its 16 chains are consecutive from
// c0 = 16 (block tpw + tile), i.e. bits c0 & 63 .. +15 of one word, set by one atomic per wave (a per-chain
// atomicOr put up to 64 device-scope atomics on every word)
__device__ __forceinline__ void glm_store_bit(const GlmArgs& a, const GlmPos& p, int64_t kk, bool acc) {
    if (a.s.order != nullptr) {                                  // permuted tile: chains anywhere, a bit each
        if (p.live && acc && p.q == 0 && p.slice == 0 && a.s.acc_bits != nullptr)
            atomicOr((unsigned long long*)&a.s.acc_bits[(size_t)kk * (size_t)a.s.nw + (size_t)(p.c >> 6)],
                     1ull << (p.c & 63));
        return;
    }
    const uint64_t m = __ballot(p.live && acc && p.q == 0 && p.slice == 0) & 0xffffull;   // lane cl < 16: bit cl
    if (p.lane == 0 && m != 0 && a.s.acc_bits != nullptr)                                   // lane 0: c == c0
        atomicOr((unsigned long long*)&a.s.acc_bits[(size_t)kk * (size_t)a.s.nw + (size_t)(p.c >> 6)],
                 (unsigned long long)(m << (p.c & 63)));
}

// normals of the lane's coordinates; padded coordinates (k >= d) get 0 so they stay at 0
template <int NM>
__device__ __forceinline__ void glm_normals(const GlmPos& p, const Stream& rs, uint32_t chain, uint32_t step,
                                            int d, double (&z)[(4 * NM)]) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
        if (true) {
            const uint32_t blk = (uint32_t)((p.base >> 2) + 4 * m + p.q);   // coords 4*blk .. 4*blk+3
            const u32x4 w = rs.block(chain, step, blk, TAG_NORMAL);
            normals4(w, z[4 * m], z[4 * m + 1], z[4 * m + 2], z[4 * m + 3]);
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if ((int)(4 * blk) + e >= d) z[4 * m + e] = 0.0;
        } else {
            z[4 * m] = z[4 * m + 1] = z[4 * m + 2] = z[4 * m + 3] = 0.0;
        }
    }
}

__device__ __forceinline__ bool glm_mh_short_circuit(const Stream& rs, uint32_t chain, uint32_t step, double ratio) {
    bool acc = ratio > 0.0;                                           // RWM.jl:63, MALA.jl:108
    if (!acc) {
        const u32x4 w = rs.block(chain, step, 0u, TAG_ACCEPT);
        acc = gt_det_log(ratio, uniform52(w.x, w.y));
    }
    return acc;
}

__device__ __forceinline__ double glm_tune_factor(int32_t acc, int32_t prop, double target) {
    const double rate = (double)acc / (double)prop;                   // MALA.jl:36-39, HMC.jl:165-169
    return 1.0 / (1.0 + det_exp(-11.0 * (rate - target))) + 0.5;
}

// ------------------------------------------------------------------ kernels
template <int NM, int NW>
__global__ __launch_bounds__(glm_block<NW>()) void glm_eval_kernel(GlmArgs a, const double* xin, double* lp_out,
                                                             double* g_out, int32_t check) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const GlmPos p = glm_pos(a);
    const GlmLds L = glm_lds(a, smem);
    double x[(4 * NM)];
    f64x4 g[NM];
    glm_load_all<NM>(a, p, xin, x);
    bool oos;
    const double lp = glm_eval<NM, NW, true>(a, p, L, x, g, oos);
    if (p.live && p.q == 0 && p.slice == 0) lp_out[p.c] = lp;
    if (g_out) glm_store4<NM>(a, p, g_out, a.s.ld, g);
    if (check && p.live && !(lp - lp == 0.0)) atomicOr(a.s.err, 1);
}

template <int NM, int NW>
__global__ __launch_bounds__(glm_block<NW>()) void glm_rwm(GlmArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const StepArgs& s = a.s;
    const GlmPos p = glm_pos(a);
    const GlmLds L = glm_lds(a, smem);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    f64x4 dummy[NM];
    const double* scl = s.scale + p.base + 4 * p.q;
    double lp = a.st.lp[p.live ? p.c : 0];
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        double xp[(4 * NM)];
        {
            double x[(4 * NM)];
            glm_load<NM>(a, p, a.st.x, x);
            glm_normals<NM>(p, rs, chain, (uint32_t)i, a.s.d, xp);
#pragma unroll
            for (int slot = 0; slot < (4 * NM); ++slot)                         // RWM.jl:59
                xp[slot] = x[slot] + xp[slot] * (glm_valid(a, p, slot) ? scl[16 * (slot >> 2) + (slot & 3)] : 0.0);
        }
        bool oos;
        const double lpp = glm_eval<NM, NW, false>(a, p, L, xp, dummy, oos);
        const bool acc = glm_mh_short_circuit(rs, chain, (uint32_t)i, lpp - lp);
        if (acc) {
            glm_store<NM>(a, p, a.st.x, s.ld, xp);
            lp = lpp;
        }
        int64_t kk;
        if (kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk)) {
            if (!acc) glm_load<NM>(a, p, a.st.x, xp);
            glm_store_kept<NM>(a, p, kk, s.samples, xp);
            glm_store_bit(a, p, kk, acc);
        }
    }
    if (p.live && p.q == 0 && p.slice == 0) a.st.lp[p.c] = lp;
    glm_count_evals(a, p, s.nsteps);
}

// RAM (RAM.jl:55-78) for d <= 32 (one d-slice, NW = 1), the factor padded to DF = 16 NM (ram.hpp).
// Row r of S belongs to the lane that owns coordinate r (own_coord): it forms u[r] = (S z)[r] from the
// full normal vector (every lane of the chain draws all DF/4 blocks), keeps it across the evaluation,
// and after the accept updates its rows of every column k; the pivot u[k] comes from its owner by a
// cross-lane read.  Rows r <= k of a column compute throw-away values whose stores go to the trash row
// of the tile (index ram_rows(DF)), so the loop carries no branches.
template <int NM, int NW>
__global__ __launch_bounds__(glm_block<NW>()) void glm_ram(GlmArgs a) {
    static_assert(NW == 1, "RAM on regression targets is built for d <= 32");
    constexpr int DF = 16 * NM;
    constexpr int NS = 4 * NM;                                          // own coordinates per lane
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const StepArgs& s = a.s;
    const GlmPos p = glm_pos(a);
    const GlmLds L = glm_lds(a, smem);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    f64x4 dummy[NM];
    // the wave's 16 chains lie in one 64-chain tile of the factor store (ram.hpp layout; padding chains past
    // the last one), addressed through buffer resources: lane offset lo, own row r's base rowb[slot]
    const uint32_t rtile = (uint32_t)__builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * a.g.tpw + p.tile) >> 2));
    double* const T0 = a.st.ram_L + (uint64_t)rtile * (uint64_t)ram_tile_doubles(DF);
    const uint64_t ld = (uint64_t)a.st.ram_ld;
    const uint32_t lo = (uint32_t)(p.c & 63) * 8;
    uint32_t rowb[NS];
#pragma unroll
    for (int slot = 0; slot < NS; ++slot) {
        const int r = own_coord(p, slot);
        rowb[slot] = lo + (uint32_t)(r * (r + 1) / 2) * 512;
    }
    const int d = s.d;
    double lp = a.st.lp[p.live ? p.c : 0];
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        double xp[NS], u[NS], nz = 0.0;
        {
            double z[DF];
#pragma unroll
            for (int b = 0; b < DF / 4; ++b) {                                  // rvec = randn(d)
                const u32x4 w = rs.block(chain, (uint32_t)i, (uint32_t)b, TAG_NORMAL);
                normals4(w, z[4 * b], z[4 * b + 1], z[4 * b + 2], z[4 * b + 3]);
            }
#pragma unroll
            for (int k = 0; k < DF; ++k) {
                if (k >= d) z[k] = 0.0;                                         // padding: identity block
                nz = __builtin_fma(z[k], z[k], nz);                             // dot(rvec, rvec)
            }
            double x[NS];
            glm_load<NM>(a, p, a.st.x, x);
            const ram_rsrc_t Rs = ram_tile_rsrc<DF>(ram_half<DF>(T0, i - 1, ld));
#pragma unroll
            for (int slot = 0; slot < NS; ++slot) {
                // own row r: the fma chain over c <= r, then exact no-ops fma(0, z, acc)
                const int r = own_coord(p, slot);
                double acc = 0.0;
#pragma unroll
                for (int c = 0; c < DF; ++c) {
                    const double v = ram_tload(Rs, rowb[slot], c);            // row r(r+1)/2 + c (in the tile)
                    acc = __builtin_fma(c <= r ? v : 0.0, z[c], acc);
                }
                u[slot] = acc;
                xp[slot] = x[slot] + acc;                                     // RAM.jl:60
                __builtin_amdgcn_sched_barrier(0);                            // one row's loads at a time
            }
        }
        bool oos;
        const double lpp = glm_eval<NM, NW, false>(a, p, L, xp, dummy, oos);
        const double ratio = lpp - lp;
        const bool acc = glm_mh_short_circuit(rs, chain, (uint32_t)i, ratio);
        if (acc) {
            glm_store<NM>(a, p, a.st.x, s.ld, xp);
            lp = lpp;
        }
        int64_t kk;
        if (kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk)) {
            if (!acc) glm_load<NM>(a, p, a.st.x, xp);
            glm_store_kept<NM>(a, p, kk, s.samples, xp);
            glm_store_bit(a, p, kk, acc);
        }
        // S <- chol(S S' + beta u u')' (ram.hpp ram_update, distributed over the chain's four lanes)
        const double beta = ram_alpha(i, d, ratio, a.sa.rate) / nz;
        const bool up = beta >= 0.0;
        const double sb = __builtin_sqrt(__builtin_fabs(beta));
#pragma unroll
        for (int slot = 0; slot < NS; ++slot) u[slot] = sb * u[slot];
        const ram_rsrc_t Rs = ram_tile_rsrc<DF>(ram_half<DF>(T0, i - 1, ld));
        const ram_rsrc_t Rd = ram_tile_rsrc<DF>(ram_half<DF>(T0, i, ld));
#pragma unroll
        for (int k = 0; k < DF; ++k) {
            const int kslot = 4 * (k >> 4) + (k & 3);                           // owner: q = (k & 15) >> 2
            const double xk = __shfl(u[kslot], p.cl + 16 * ((k & 15) >> 2), 64);
            const double lkk = ram_tload(Rs, lo, k * (k + 1) / 2 + k);
            const double t2 = xk * xk;
            const double l2 = lkk * lkk;
            const double r = __builtin_sqrt(up ? l2 + t2 : l2 - t2);
            const double cc = r / lkk;
            const double sn = xk / lkk;
            const double sns = up ? sn : -sn;                                   // as ram.hpp ram_update
            const double ic = 1.0 / cc;
            ram_tstore(Rd, lo, k * (k + 1) / 2 + k, r);
#pragma unroll
            for (int slot = 0; slot < NS; ++slot) {
                const int q = own_coord(p, slot);
                if (16 * (slot >> 2) + 12 + (slot & 3) <= k) continue;          // no row of this slot is below k
                const bool below = q > k;
                const double l0 = ram_tload(Rs, rowb[slot], k);                // in bounds for q <= k too
                const double l = (l0 + sns * u[slot]) * ic;
                // rows q <= k store to the tile's trash row (index ram_rows(DF))
                ram_tstore(Rd, below ? rowb[slot] : lo + (uint32_t)(ram_rows(DF) - k) * 512, k, l);
                const double un = cc * u[slot] - sn * l;
                u[slot] = below ? un : u[slot];
            }
            __builtin_amdgcn_sched_barrier(0);                                  // one column's loads at a time
        }
    }
    if (p.live && p.q == 0 && p.slice == 0) a.st.lp[p.c] = lp;
    glm_count_evals(a, p, s.nsteps);
}

template <int NM, int NW>
__global__ __launch_bounds__(glm_block<NW>()) void glm_mala(GlmArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const GlmPos p = glm_pos(a);
    const GlmLds L = glm_lds(a, smem);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    const int64_t cc = p.live ? p.c : 0;
    double lp = a.st.lp[cc];
    double h = sa.tuner ? a.st.t_step[cc] : sa.drift_step;
    int32_t n_acc = sa.tuner ? a.st.t_acc[cc] : 0;
    int32_t n_prop = sa.tuner ? a.st.t_prop[cc] : 0;
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        if (sa.tuner) n_prop += 1;
        const double half = h / 2.0;
        const double sq = __builtin_sqrt(h);
        const double twoh = 2.0 * h;
        const double Lc = det_log(kTwoPi * h) / 2.0;
        double xp[(4 * NM)];
        f64x4 gp[NM];
        double qf = 0.0;
        {
            double x[(4 * NM)];                                        // state, reloaded after eval
            glm_normals<NM>(p, rs, chain, (uint32_t)i, a.s.d, xp);
            glm_load<NM>(a, p, a.st.x, x);
            glm_load4<NM>(a, p, a.st.g, gp);                           // current gradient (state)
#pragma unroll
            for (int slot = 0; slot < (4 * NM); ++slot) {
                const double pm = x[slot] + half * gp[slot >> 2][slot & 3];   // MALA.jl:98
                xp[slot] = pm + sq * xp[slot];                                 // MALA.jl:100
                const double e = pm - xp[slot];
                if (glm_valid(a, p, slot)) qf = qf + ((-(e * e)) / twoh - Lc);   // MALA.jl:103
            }
        }
        qf = glm_sum(a, p, L, qf);
        bool oos;
        const double lpp = glm_eval<NM, NW, true>(a, p, L, xp, gp, oos);    // MALA.jl:101
        double qb = 0.0;
        {
            double x[(4 * NM)];
            glm_load<NM>(a, p, a.st.x, x);
#pragma unroll
            for (int slot = 0; slot < (4 * NM); ++slot) {
                const double e = (xp[slot] + half * gp[slot >> 2][slot & 3]) - x[slot];   // MALA.jl:104-105
                if (glm_valid(a, p, slot)) qb = qb + ((-(e * e)) / twoh - Lc);
            }
        }
        qb = glm_sum(a, p, L, qb);
        const double ratio = ((lpp + qb) - lp) - qf;                   // MALA.jl:107
        const bool acc = glm_mh_short_circuit(rs, chain, (uint32_t)i, ratio);
        if (acc) {
            glm_store<NM>(a, p, a.st.x, s.ld, xp);
            glm_store4<NM>(a, p, a.st.g, s.ld, gp);
            lp = lpp;
            if (sa.tuner) n_acc += 1;
        }
        int64_t kk;
        if (kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk)) {
            if (!acc) {
                glm_load<NM>(a, p, a.st.x, xp);
                glm_load4<NM>(a, p, a.st.g, gp);
            }
            glm_store_kept<NM>(a, p, kk, s.samples, xp);
            glm_store_kept4<NM>(a, p, kk, s.grads, gp);
            glm_store_bit(a, p, kk, acc);
        }
        if (sa.tuner && i <= s.tuner_burnin && (i % sa.adapt_step) == 0) {   // MALA.jl:116-118
            h = h * glm_tune_factor(n_acc, n_prop, sa.target_rate);
            n_acc = 0;
            n_prop = 0;
        }
    }
    if (p.live && p.q == 0 && p.slice == 0) {
        a.st.lp[p.c] = lp;
        if (sa.tuner) {
            a.st.t_step[p.c] = h;
            a.st.t_acc[p.c] = n_acc;
            a.st.t_prop[p.c] = n_prop;
        }
    }
    glm_count_evals(a, p, s.nsteps);
}

// MALA on one slice (d <= 128): as glm_mala, with the proposal kept in the lane's private LDS slots
// (L.beta) instead of registers -- built block by block from the normals and the state in HBM, read by
// the eta MFMAs as their B operands and by the backward density afterwards -- so that only the
// gradient accumulators live across the tile loop.  One launch is one step: inside a step loop the
// compiler hoists the tile loop's invariant addresses and constants out of it and the kernel spills
// (> 512 registers); the per-chain scalars (lp, tuner state) round-trip through HBM per launch instead.
// Same operations in the same order as glm_mala.
template <int NM>
__global__ __launch_bounds__(glm_block<1>()) void glm_mala1(GlmArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int NS = 4 * NM;
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const GlmPos p = glm_pos(a);
    const GlmLds L = glm_lds(a, smem);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    const int64_t cc = p.live ? p.c : 0;
    double* const xb = L.beta + (size_t)(p.wave * NS) * 64 + p.lane;
    const size_t ld = (size_t)s.ld;
    const double* const xl = glm_lane_ptr(p, a.st.x, s.ld, cc);
    const double* const gl = glm_lane_ptr(p, a.st.g, s.ld, cc);
    double lp = a.st.lp[cc];
    double h = sa.tuner ? a.st.t_step[cc] : sa.drift_step;
    int32_t n_acc = sa.tuner ? a.st.t_acc[cc] : 0;
    int32_t n_prop = sa.tuner ? a.st.t_prop[cc] : 0;
    {                                   // ONE step per launch (mcmc_glm_steps_per_launch): no step loop
        const int t = 0;
        const int64_t i = s.step_begin + t;
        if (sa.tuner) n_prop += 1;
        const double half = h / 2.0;
        const double sq = __builtin_sqrt(h);
        const double twoh = 2.0 * h;
        const double Lc = det_log(kTwoPi * h) / 2.0;
        double qf = 0.0;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const uint32_t blk = (uint32_t)((p.base >> 2) + 4 * m + p.q);      // coords 4*blk .. 4*blk+3
            const u32x4 w = rs.block(chain, (uint32_t)i, blk, TAG_NORMAL);
            double z[4];
            normals4(w, z[0], z[1], z[2], z[3]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int slot = 4 * m + e;
                const bool v = glm_valid(a, p, slot);
                const size_t o = (size_t)(16 * m + e) * ld;
                const double xv = v ? xl[o] : 0.0;
                const double gv = v ? gl[o] : 0.0;
                const double pm = xv + half * gv;                               // MALA.jl:98
                const double xpv = pm + sq * (v ? z[e] : 0.0);                  // MALA.jl:100
                const double ee = pm - xpv;
                if (v) qf = qf + ((-(ee * ee)) / twoh - Lc);                    // MALA.jl:103
                xb[64 * slot] = xpv;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        qf = glm_sum(a, p, L, qf);
        bool oos;
        f64x4 gp[NM];
        const double lpp = glm_eval1<NM, true>(a, p, L, XLds{xb}, gp, oos);    // MALA.jl:101
        double qb = 0.0;
#pragma unroll
        for (int slot = 0; slot < NS; ++slot) {
            const bool v = glm_valid(a, p, slot);
            const double xv = v ? xl[(size_t)(16 * (slot >> 2) + (slot & 3)) * ld] : 0.0;
            const double e = (xb[64 * slot] + half * gp[slot >> 2][slot & 3]) - xv;   // MALA.jl:104-105
            if (v) qb = qb + ((-(e * e)) / twoh - Lc);
        }
        qb = glm_sum(a, p, L, qb);
        const double ratio = ((lpp + qb) - lp) - qf;                   // MALA.jl:107
        const bool acc = glm_mh_short_circuit(rs, chain, (uint32_t)i, ratio);
        int64_t kk;
        const bool kept = kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk);
        double* const ks = kept && s.samples ? s.samples + (size_t)kk * (size_t)s.d * (size_t)s.C : nullptr;
        double* const kg = kept && s.grads ? s.grads + (size_t)kk * (size_t)s.d * (size_t)s.C : nullptr;
        if (p.live) {
            double* const xw = a.st.x + (size_t)(p.base + 4 * p.q) * ld + (size_t)p.c;
            double* const gw = a.st.g + (size_t)(p.base + 4 * p.q) * ld + (size_t)p.c;
            const size_t Cs = (size_t)s.C;
#pragma unroll
            for (int slot = 0; slot < NS; ++slot) {
                if (!glm_valid(a, p, slot)) continue;
                const size_t r = (size_t)(16 * (slot >> 2) + (slot & 3));
                double xv, gv;
                if (acc) {
                    xv = xb[64 * slot];
                    gv = gp[slot >> 2][slot & 3];
                    xw[r * ld] = xv;
                    gw[r * ld] = gv;
                } else {
                    xv = xl[r * ld];
                    gv = gl[r * ld];
                }
                const size_t ko = (size_t)(p.base + 4 * p.q + r) * Cs + (size_t)p.c;
                if (ks) ks[ko] = xv;
                if (kg) kg[ko] = gv;
            }
        }
        if (acc) {
            lp = lpp;
            if (sa.tuner) n_acc += 1;
        }
        if (kept) glm_store_bit(a, p, kk, acc);
        if (sa.tuner && i <= s.tuner_burnin && (i % sa.adapt_step) == 0) {   // MALA.jl:116-118
            h = h * glm_tune_factor(n_acc, n_prop, sa.target_rate);
            n_acc = 0;
            n_prop = 0;
        }
    }
    if (p.live && p.q == 0 && p.slice == 0) {
        a.st.lp[p.c] = lp;
        if (sa.tuner) {
            a.st.t_step[p.c] = h;
            a.st.t_acc[p.c] = n_acc;
            a.st.t_prop[p.c] = n_prop;
        }
    }
    glm_count_evals(a, p, s.nsteps);
}

// ------------------------------------------------------------------ batched proposal normals
// normals4 (detmath.hpp) of NB Philox blocks, bitwise -- the same operations on the same values -- with every
// table-row load of the 2 NB radii (bm_radius_u32's main rows) and the 2 NB angles (det_sincos2pi_u32's row) issued
// before the first is used.  normals4 waits for each radius's rows in turn, and the radius tail branch waits for
// every load in flight, so a wave drawing a 128-coordinate proposal from the global tables paid about four memory
// latencies per block; here the rows of all NB blocks are in flight together and only a (rare, 2^-11 per draw) tail
// lane costs a wait of its own.
template <int NB>
__device__ __forceinline__ void normals_batch(const u32x4 (&w)[NB], double (&z)[4 * NB]) {
    typedef double f64x2_t __attribute__((ext_vector_type(2)));
    constexpr int NR = 2 * NB;
    constexpr uint32_t kOff0 = 0u - ((uint32_t)((1023 + 21) << 5) << 4);
    constexpr uint32_t kOff1 = kOff0 + (uint32_t)(BM_RADP_NROWS / 2) * 16u;
    uint32_t wr[NR], wa[NR];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        wr[2 * b] = w[b].x; wa[2 * b] = w[b].y;
        wr[2 * b + 1] = w[b].z; wa[2 * b + 1] = w[b].w;
    }
    uint32_t vv[NR], smv[NR];
    bool tl[NR];
    double t[NR];
    f64x2_t c[NR][4];
#pragma unroll
    for (int k = 0; k < NR; ++k) {                                      // bm_radius_u32: the main-table rows
        const uint32_t sm = (uint32_t)((int32_t)wr[k] >> 31);
        const uint32_t v = wr[k] ^ sm;
        const double y = (double)v;
        const uint64_t b = d2bits(y);
        const uint32_t yh = (uint32_t)(b >> 32);
        tl[k] = v < (1u << 21);
        const uint32_t sel = (sm & kOff1) | (~sm & kOff0);
        uint32_t off = ((yh >> 15) << 4) + sel;
        const uint32_t th = (yh & 0x7fffu) | 0x3ff00000u;
        off = tl[k] ? 0u : off;
        t[k] = bits2d(((uint64_t)th << 32) | (b & 0xffffffffull)) - (1.0 + 1.0 / 64.0);
        const char* base = reinterpret_cast<const char*>(kBmRadPTab) + off;
        c[k][0] = *reinterpret_cast<const f64x2_t*>(base);
        c[k][1] = *reinterpret_cast<const f64x2_t*>(base + 16 * BM_RADP_NROWS);
        c[k][2] = *reinterpret_cast<const f64x2_t*>(base + 32 * BM_RADP_NROWS);
        c[k][3] = *reinterpret_cast<const f64x2_t*>(base + 48 * BM_RADP_NROWS);
        vv[k] = v;
        smv[k] = sm;
    }
    int32_t ji[NR];
    f64x2_t ar[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {                                      // det_sincos2pi_u32: the (sin a, cos a) row
        ji[k] = ((int32_t)(wa[k] << 10)) >> 10;
        const uint32_t off = (wa[k] - (uint32_t)ji[k]) >> 18;
        ar[k] = *reinterpret_cast<const f64x2_t*>(reinterpret_cast<const char*>(kBmSinCos1024Tab) + off);
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {                                      // bm_radius_u32's tail, on the lanes in it
        if (tl[k]) {
            uint32_t v2 = vv[k];
            asm volatile("" : "+v"(v2));
            const double x = (double)v2 + 0.5;
            const uint64_t bx = d2bits(x);
            const uint32_t xh = (uint32_t)(bx >> 32);
            const uint32_t rw = (uint32_t)((int)(xh >> 15) - ((1023 - 1) << 5)) * 16u +
                                (smv[k] & (16u * (BM_RADT_NROWS / 2)));
            t[k] = bits2d(((uint64_t)((xh & 0x7fffu) | 0x3ff00000u) << 32) | (bx & 0xffffffffull)) - (1.0 + 1.0 / 64.0);
            asm volatile(
                "global_load_dwordx4 %0, %4, %5\n\t"
                "global_load_dwordx4 %1, %4, %6\n\t"
                "global_load_dwordx4 %2, %4, %7\n\t"
                "global_load_dwordx4 %3, %4, %8\n\t"
                "s_waitcnt vmcnt(0)"
                : "=&v"(c[k][0]), "=&v"(c[k][1]), "=&v"(c[k][2]), "=&v"(c[k][3])
                : "v"(rw), "s"(&kBmRadTTab[0][0]), "s"(&kBmRadTTab[BM_RADT_NROWS][0]),
                  "s"(&kBmRadTTab[2 * BM_RADT_NROWS][0]), "s"(&kBmRadTTab[3 * BM_RADT_NROWS][0])
                : "memory");
        }
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        double q = __builtin_fma(c[k][3].y, t[k], c[k][3].x);           // the radius polynomial
        q = __builtin_fma(q, t[k], c[k][2].y);
        q = __builtin_fma(q, t[k], c[k][2].x);
        q = __builtin_fma(q, t[k], c[k][1].y);
        q = __builtin_fma(q, t[k], c[k][1].x);
        q = __builtin_fma(q, t[k], c[k][0].y);
        const double rad = __builtin_fma(q, t[k], c[k][0].x);
        const double j = (double)ji[k];                                 // the angle
        const double j2 = j * j;
        const double sr = j * __builtin_fma(j2, __builtin_fma(j2, kSinJ5, kSinJ3), kSinJ1);
        const double cr = __builtin_fma(j2, __builtin_fma(j2, kCosJ4, kCosJ2), 1.0);
        const double sn = __builtin_fma(ar[k].x, cr, ar[k].y * sr);
        const double cs = __builtin_fma(ar[k].y, cr, -(ar[k].x * sr));
        z[2 * k] = rad * cs;
        z[2 * k + 1] = rad * sn;
    }
}

// ------------------------------------------------------------------ wave-specialised single-slice MALA
// glm_mala1ws<NM>: glm_mala1's step (config 3: logistic MALA, d = 128) with the work of a 16-chain tile split over
// two waves that share a SIMD (a 512-thread workgroup puts waves w and w + 4 on one SIMD):
//   wave w < 4   ("M", matrix): holds the tile's proposal (the B operands) and the gradient accumulators in registers
//                and issues every MFMA: eta_{t+1} = X_{t+1} beta and G += X_{t-1}^T r_{t-1};
//   wave w + 4   ("V", vector): the proposal (Philox, Box-Muller, MALA.jl:98-103), the X tile loads and, per
//                observation tile, the elementwise log-likelihood terms and residual weights r_t on eta_t.
// eta_t and r_t cross through LDS (double-buffered), one barrier per tile.  The fp64 matrix and vector pipes of a
// SIMD run concurrently for different waves (scripts/peak_f64.hip: MFMA-only and FMA-only waves paired on a SIMD
// take max, not sum, of their times), whereas glm_mala1's single wave per SIMD (300 VGPRs) serialises its VALU
// work with its MFMAs.  Every sum is formed by the same instructions in the same order as glm_mala1 (eta chains
// over (m, e, q); G chains over observations; a lane's likelihood terms in (t, r) order; qf / qb / prior as
// there), so the results are glm_mala1's bit for bit and orc_glm_eval restates them.
// LDS (doubles; XS = glm_tile_doubles(16 NM), X rows then Y): X slots 0, 1 | region R: X slots 2, 3, eta [2][4][64][4], r [2][4][64][4],
// which overlays the proposal [4 waves][4 NM][64] of the proposal phase | Y [4][16] | the logistic term's table
// (kSoftplusTab) | qf, lik [2][4][16] | M's partial qf [4][64].
template <int NM>
__host__ __device__ constexpr int glm_ws_region(int XS) {
    return (2 * XS + 4096) > (4 * 4 * NM * 64) ? (2 * XS + 4096) : (4 * 4 * NM * 64);
}
__host__ __device__ inline size_t glm_ws_lds_doubles(int nm) {
    const int XS = glm_tile_doubles(16 * nm);
    const int R = (2 * XS + 4096) > (4 * 4 * nm * 64) ? (2 * XS + 4096) : (4 * 4 * nm * 64);
    return (size_t)(2 * XS + R + 4 * 16 + SP_NROWS * 10 + 2 * 4 * 16 + 4 * 64)
#ifdef GLM_WS_STAMP
           + 512                                               // the phase stamps (dev build, scripts/ws_stamps.py)
#endif
        ;
}
#ifdef GLM_WS_STAMP
// GLM_WS_STAMP (dev build only, scripts/ws_stamps.py): shader-clock stamps (low 32 bits) of glm_mala1ws's tile loop,
// every wave of workgroups 0..3, tiles 8..23: M waves at the loop top, eta_{t+1} stored, G_{t-1} issued, past the
// barrier; V waves at the loop top, tile t+2 stored / t+3 issued, the terms of tile t done, r_t stored, past the
// barrier.  Kept in LDS past the kernel's own and copied out after the loop.
static __device__ unsigned g_ws_stamps[4][8][16][8];
static __device__ unsigned g_ws_wg[4][8][8];           // per wave: start, proposal, bx/tile 2, eta_0, loop end, final barrier, end
static __device__ unsigned g_ws_wg2[4][8][8];          // inside the proposal phase (V: normals done, qf summed, table; M: tiles 0, 1)
#define WS_WG2(pt)                                                                                     \
    do {                                                                                               \
        const unsigned ts_ = (unsigned)__builtin_amdgcn_s_memtime();                                  \
        if (blockIdx.x < 4 && (threadIdx.x & 63) == 0) g_ws_wg2[blockIdx.x][threadIdx.x >> 6][pt] = ts_; \
    } while (0)
#define WS_WG(pt)                                                                                      \
    do {                                                                                               \
        const unsigned ts_ = (unsigned)__builtin_amdgcn_s_memtime();                                  \
        if (blockIdx.x < 4 && (threadIdx.x & 63) == 0) g_ws_wg[blockIdx.x][threadIdx.x >> 6][pt] = ts_; \
    } while (0)
#define WS_STAMP(pt)                                                                                   \
    do {                                                                                               \
        if (t >= 8 && t < 24) {                                                                        \
            const unsigned ts_ = (unsigned)__builtin_amdgcn_s_memtime();                              \
            if (p.lane == 0) wst[(wv * 16 + (int)(t - 8)) * 8 + (pt)] = ts_;                          \
        }                                                                                              \
    } while (0)
#else
#define WS_STAMP(pt) do { } while (0)
#define WS_WG(pt) do { } while (0)
#define WS_WG2(pt) do { } while (0)
#endif
template <int NM, bool UNITP = false>
__global__ __launch_bounds__(512) void glm_mala1ws(GlmArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int NS = 4 * NM;
    constexpr int KM = 4 * NM;
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const ModelArgs& M = a.m;
    const GlmShape& g = a.g;
    const int wv = (int)(threadIdx.x >> 6);
    const bool vwave = __builtin_amdgcn_readfirstlane(wv) >= 4;
    GlmPos p;
    p.lane = threadIdx.x & 63;
    p.q = p.lane >> 4;
    p.cl = p.lane & 15;
    p.tile = wv & 3;
    p.wave = p.tile;
    p.slice = 0;
    p.base = 0;
    p.c = ((int64_t)blockIdx.x * 4 + p.tile) * 16 + p.cl;
    p.live = p.c < s.C;
    constexpr int S = glm_row_stride(16 * NM);
    constexpr int XS = glm_tile_doubles(16 * NM);             // one staged tile: X rows, then Y
    constexpr int YO = glm_y_offset(16 * NM);
    constexpr int BO = glm_b_offset(16 * NM);
    double* const Xs = smem;                                   // 4 X tile slots: 0, 1 here, 2, 3 in region R
    double* const R = smem + 2 * XS;
    double* const Eb = R + 2 * XS;                             // eta [2][4 tiles][64 lanes][4]
    double* const Rb = Eb + 2048;                              // r   [2][4 tiles][64 lanes][4]
    double* const beta = R;                                    // proposal [4 tiles][NS][64] (proposal phase only)
    double* const Yb = R + glm_ws_region<NM>(XS);              // (unused: Y travels inside each staged tile)
    double* const ltabp = Yb + 64;                             // logistic term's table [SP_NROWS][10]
    double* const qfl = ltabp + SP_NROWS * 10;                 // qf [4][16], then lik [4][16]
    double* const likl = qfl + 64;
    double* const qpart = likl + 64;                           // M's partial qf per lane [4 tiles][64] (proposal phase)
#ifdef GLM_WS_STAMP
    unsigned* const wst = reinterpret_cast<unsigned*>(qpart + 256);
#endif
    auto xslot = [&](int64_t tt) -> double* { const int b = (int)(tt & 3); return b < 2 ? Xs + b * XS : R + (b - 2) * XS; };
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    const int64_t cc = p.live ? p.c : 0;
    const size_t ld = (size_t)s.ld;
    const double* const xl = glm_lane_ptr(p, a.st.x, s.ld, cc);
    const double* const gl = glm_lane_ptr(p, a.st.g, s.ld, cc);
    const int64_t i = s.step_begin;                            // ONE step per launch (as glm_mala1)
    const double h = sa.tuner ? a.st.t_step[cc] : sa.drift_step;
    const double half = h / 2.0;
    const double twoh = 2.0 * h;
    const double Lc = det_log(kTwoPi * h) / 2.0;
    const int64_t ntiles = g.n_pad / 16;
    const bool logi = M.kind == MK_LOGISTIC;
    // X / Y tile transfer, by the 256 threads of one wave role (u = thread index within the role)
    constexpr int kHalf = XS / 2;                              // f64x2 per staged tile
    constexpr int kPer = (kHalf + 255) / 256;
    const int u = (int)(threadIdx.x & 255);
    f64x2 xbuf[kPer];
    (void)Yb;
    auto load_tile = [&](int64_t tt) {                         // the tile image moves linearly (glm_layout.hpp)
        const f64x2* src = reinterpret_cast<const f64x2*>(M.X + (size_t)tt * XS);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int e = u + 256 * j;
            xbuf[j] = src[e < kHalf ? e : 0];
        }
    };
    auto store_tile = [&](int64_t tt) {
        f64x2* dst = reinterpret_cast<f64x2*>(xslot(tt));
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int e = u + 256 * j;
            if (e < kHalf) dst[e] = xbuf[j];
        }
    };
    double* const xb = beta + (size_t)(p.tile * NS) * 64 + p.lane;   // this lane's proposal slots

    // ---- proposal phase: the proposal (MALA.jl:98-103) into LDS, its Philox blocks split between the tile's two
    //      waves (M: m < NM/2, V: the rest; the proposal is latency-bound -- table reads, state loads -- and the M
    //      waves had only the X tiles 0 and 1 to stage); qf's sum runs in slot order: M's partial over its slots
    //      crosses to V through LDS and V continues it over its own, so the sum is glm_mala1's
    WS_WG(0);
    constexpr int m_split = NM / 2;
    double tv[NS];                                             // V: its slots' qf terms, summed after M's partial
    {
        double qf = 0.0;
        const double sq = __builtin_sqrt(h);
        // the wave's blocks [M0, M1): the blocks' normals with their table rows in flight together, then the state
        // (every load unconditional: an invalid slot reads the chain's row 0 and is zeroed)
        auto part = [&](auto m0c, auto m1c) {
            constexpr int M0 = decltype(m0c)::value, M1 = decltype(m1c)::value, NBK = M1 - M0;
            if constexpr (NBK > 0) {
                u32x4 w[NBK];
#pragma unroll
                for (int b = 0; b < NBK; ++b)                                  // coords 4*blk .. 4*blk+3
                    w[b] = rs.block(chain, (uint32_t)i, (uint32_t)(4 * (M0 + b) + p.q), TAG_NORMAL);
                double z[4 * NBK];
                normals_batch<NBK>(w, z);
#pragma unroll
                for (int k = 0; k < 4 * NBK; ++k) {
                    const int slot = 4 * M0 + k;
                    const bool v = glm_valid(a, p, slot);
                    const ptrdiff_t o = glm_slot_off(a, p, slot, ld);
                    // global loads (as flat loads, each LDS store of the proposal below would wait for them all)
                    typedef const __attribute__((address_space(1))) double gdouble;
                    const double xl0 = *(gdouble*)(xl + o), gl0 = *(gdouble*)(gl + o);
                    const double xv = v ? xl0 : 0.0;
                    const double gv = v ? gl0 : 0.0;
                    const double pm = xv + half * gv;                           // MALA.jl:98
                    const double xpv = pm + sq * (v ? z[k] : 0.0);              // MALA.jl:100
                    const double ee = pm - xpv;
                    const double term = (-(ee * ee)) / twoh - Lc;               // MALA.jl:103
                    if (vwave) tv[slot] = term;
                    else if (v) qf = qf + term;
                    xb[64 * slot] = xpv;
                }
            }
        };
        if (vwave) part(std::integral_constant<int, NM / 2>{}, std::integral_constant<int, NM>{});
        else part(std::integral_constant<int, 0>{}, std::integral_constant<int, NM / 2>{});
        WS_WG2(0);
        if (!vwave) qpart[p.tile * 64 + p.lane] = qf;
    }
    if (vwave) {
        if (logi) {
            for (int e = u; e < SP_NROWS * 10; e += 256) ltabp[e] = (&kSoftplusTab[0][0])[e];
        }
        WS_WG2(1);
    } else {
        load_tile(0);
        store_tile(0);
        if (ntiles > 1) {
            load_tile(1);
            store_tile(1);
        }
        WS_WG2(1);
    }
    __syncthreads();
    WS_WG(1);
    // ---- M: the proposal into registers, eta_0;  V: qf, X tile 2 into registers (slot 2 overlays the proposal)
    double bx[NS];
    f64x4 G[NM];
    if (!vwave) {
#pragma unroll
        for (int slot = 0; slot < NS; ++slot) bx[slot] = xb[64 * slot];
#pragma unroll
        for (int T = 0; T < NM; ++T) G[T] = f64x4{0.0, 0.0, 0.0, 0.0};
    } else {
        double qf = qpart[p.tile * 64 + p.lane];
#pragma unroll
        for (int slot = 4 * m_split; slot < NS; ++slot)
            if (glm_valid(a, p, slot)) qf = qf + tv[slot];
        qf = glm_sum(a, p, GlmLds{}, qf);
        if (p.q == 0) qfl[p.tile * 16 + p.cl] = qf;
        WS_WG2(2);
        if (!GLM_WS_DMA && ntiles > 2) load_tile(2);
    }
    __syncthreads();                                           // the proposal area is free from here on
    WS_WG(2);
    f64x4* const Eq = reinterpret_cast<f64x4*>(Eb) + p.tile * 64 + p.lane;   // + 256 * buffer
    f64x4* const Rq = reinterpret_cast<f64x4*>(Rb) + p.tile * 64 + p.lane;
    auto eta_of = [&](int64_t tt) {                            // glm_eval1_tiles' eta chain, operands read ahead
        const double* xrow = xslot(tt) + p.cl * S + 4 * p.q;
        constexpr int kLA = GLM_WS_LA;
        double av[KM];
#pragma unroll
        for (int m = 0; m < (kLA < KM ? kLA : KM); ++m) av[m] = xrow[glm_eta_off(m)];
        f64x4 e = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            if (m + kLA < KM) av[m + kLA] = xrow[glm_eta_off(m + kLA)];
            e = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m], bx[m], e, 0, 0, 0);
        }
        return e;
    };
    auto g_of = [&](int64_t tt) {                              // G += X_tt^T r_tt (glm_eval1_tiles' G product)
        const f64x4 rv = Rq[256 * (tt & 1)];
        const double* gcol = xslot(tt) + p.q * S + 4 * (p.cl & 3) + (p.cl >> 2);
        double ga[NM];
#pragma unroll
        for (int T = 0; T < NM; ++T) ga[T] = gcol[glm_g_off(T)];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            double gn[NM];
            if (kk < 3) {
#pragma unroll
                for (int T = 0; T < NM; ++T) gn[T] = gcol[4 * (kk + 1) * S + glm_g_off(T)];
            }
#pragma unroll
            for (int T = 0; T < NM; ++T) G[T] = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[T], rv[kk], G[T], 0, 0, 0);
            if (kk < 3) {
#pragma unroll
                for (int T = 0; T < NM; ++T) ga[T] = gn[T];
            }
        }
    };
    if (!vwave) Eq[0] = eta_of(0);
    __syncthreads();
    WS_WG(3);
    // ---- the observation tiles
    const double sn = M.noise_sigma, s2n = sn * sn;
    const double logsn = logi ? 0.0 : det_log(sn);
    const double isn = 1.0 / sn, is2n = 1.0 / s2n;
    const double (*sptab)[10] = reinterpret_cast<const double (*)[10]>(ltabp);
    const int64_t nfull = M.n / 16;
    // one loop per role, each with one barrier per tile (the same count): the roles' loop invariants (the V waves'
    // polynomial constants, the M waves' operand addresses) stay out of each other's register pressure
    double lik_part = 0.0;
    double ubnd = -__builtin_inf();                            // logistic: max of u + b over the lane's observations
    if (!vwave) {
        for (int64_t t = 0; t < ntiles; ++t) {
            WS_STAMP(0);
            if (t + 1 < ntiles) Eq[256 * ((t + 1) & 1)] = eta_of(t + 1);
            WS_STAMP(1);
            if (t >= 1) g_of(t - 1);
            WS_STAMP(2);
            __syncthreads();
            WS_STAMP(3);
        }
    } else {
        for (int64_t t = 0; t < ntiles; ++t) {
            WS_STAMP(0);
            if (t + 2 < ntiles) {                              // slot (t+2) % 4 held tile t-2: read before the last barrier
                if (GLM_WS_DMA) {
                    glm_dma_tile_w<XS, 4>(M.X + (size_t)(t + 2) * XS, xslot(t + 2), __builtin_amdgcn_readfirstlane(wv - 4));
                } else {
                    store_tile(t + 2);
                    if (t + 3 < ntiles) load_tile(t + 3);
                }
            }
            WS_STAMP(1);
            const f64x4 eta = Eq[256 * (t & 1)];
            const double* LY = xslot(t) + YO;
            double y[4], term[4], rv[4];                       // y: the response, for the logistic model w (det_logi)
#pragma unroll
            for (int r = 0; r < 4; ++r) y[r] = LY[p.q + 4 * r];
            if (logi) {
                // prob = 1/(1+exp(-X*vars)); Y ~ Bernoulli(prob); its eta-derivative (MCMCDerivRules.jl:111)
                const double* LB = xslot(t) + BO;
                // two rows at a time: four rows' coefficient rows in flight at once spill the wave's registers
#pragma unroll
                for (int h = 0; h < 4; h += 2) {
                    LogiState E[2];
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        det_logi_s1(eta[h + r], y[h + r], E[r], sptab);
                        ubnd = __builtin_fmax(ubnd, E[r].u + LB[p.q + 4 * (h + r)]);   // the reference's -Inf
                    }
#pragma unroll
                    for (int r = 0; r < 2; ++r) det_logi_s2(E[r]);
#pragma unroll
                    for (int r = 0; r < 2; ++r) det_logi_fin(E[r], y[h + r], term[h + r], rv[h + r]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            } else if (M.kind == MK_PROBIT) {
#pragma unroll
                for (int r = 0; r < 4; ++r) glm_probit_obs(eta[r], y[r], term[r], rv[r]);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double resid = y[r] - eta[r];                            // resid = Y - X*vars
                    const double zz = resid * isn;
                    term[r] = -0.5 * (zz * zz + kLog2Pi) - logsn;                  // resid ~ Normal(0, sn)
                    rv[r] = resid * is2n;
                }
            }
            if (t < nfull) {                                                       // uniform: no padded observation
#pragma unroll
                for (int r = 0; r < 4; ++r) lik_part = lik_part + term[r];         // the lane's terms in (t, r) order
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const bool in = t * 16 + p.q + 4 * r < M.n;
                    lik_part = in ? lik_part + term[r] : lik_part;
                    rv[r] = in ? rv[r] : 0.0;
                }
            }
            WS_STAMP(2);
            Rq[256 * (t & 1)] = f64x4{rv[0], rv[1], rv[2], rv[3]};
            WS_STAMP(3);
            if (GLM_WS_DMA) glm_dma_wait();                    // tile t+2 landed (the asm loads are not counted)
            __syncthreads();
            WS_STAMP(4);
        }
    }
    WS_WG(4);
#ifdef GLM_WS_STAMP
    if (blockIdx.x < 4)
        for (int j = p.lane; j < 128; j += 64) (&g_ws_stamps[blockIdx.x][wv][0][0])[j] = wst[wv * 128 + j];
#endif
    if (vwave) {
        const double lik = glm_sum(a, p, GlmLds{}, logi && ubnd >= 0.0 ? -__builtin_inf() : lik_part);
        if (p.q == 0) likl[p.tile * 16 + p.cl] = lik;
    } else {
        g_of(ntiles - 1);
    }
    __syncthreads();
    WS_WG(5);
    if (vwave) return;
    // ---- M waves: the end of the evaluation (glm_finish), MALA.jl:104-125
    // the current position (qb, and the kept rows of a rejected step), every load unconditional and issued first
    typedef const __attribute__((address_space(1))) double gdouble;   // global, not flat, loads (see the proposal)
    double xo[NS];
#pragma unroll
    for (int slot = 0; slot < NS; ++slot)
        xo[slot] = *(gdouble*)(xl + glm_slot_off(a, p, slot, ld));
    double lp = a.st.lp[cc];
    int32_t n_acc = sa.tuner ? a.st.t_acc[cc] : 0;
    int32_t n_prop = sa.tuner ? a.st.t_prop[cc] : 0;
    if (sa.tuner) n_prop += 1;
    const double qf = qfl[p.tile * 16 + p.cl];
    bool oos;
    double lpp;
    {
        const int d = M.d;
        const double lik = likl[p.tile * 16 + p.cl];
        const double sp = M.prior_sigma, s2p = sp * sp, logsp = det_log(sp);
        // the prior's divisions by sigma and sigma^2 (vars ~ Normal(0, sigma)) are exact no-ops at sigma = 1 (the
        // examples' prior, x / 1 == x for every double): the UNITP instance (launched when prior_sigma == 1) skips
        // them, bitwise the same (64 IEEE divisions a lane, a third of this phase)
        constexpr bool unit = UNITP;
        double pp = 0.0;
        if (unit) {
#pragma unroll
            for (int slot = 0; slot < NS; ++slot) {
                const int k = own_coord(p, slot);
                if (k < d) {
                    const double z = bx[slot] - 0.0;
                    pp = pp + (-0.5 * (z * z + kLog2Pi) - logsp);
                }
            }
        } else {
#pragma unroll
            for (int slot = 0; slot < NS; ++slot) {
                const int k = own_coord(p, slot);
                if (k < d) {
                    const double z = (bx[slot] - 0.0) / sp;
                    pp = pp + (-0.5 * (z * z + kLog2Pi) - logsp);
                }
            }
        }
        const double prior = glm_sum(a, p, GlmLds{}, pp);
        double acc = 0.0 + prior;                                           // LLAcc(0.) + ...
        bool bad = !(acc - acc == 0.0);
        acc = acc + lik;
        bad = bad || !(acc - acc == 0.0);
        oos = bad;
        if (bad) acc = -__builtin_inf();
        if (unit) {
#pragma unroll
            for (int slot = 0; slot < NS; ++slot)
                G[slot >> 2][slot & 3] = bad ? 0.0 : (0.0 - bx[slot]) + G[slot >> 2][slot & 3];
        } else {
#pragma unroll
            for (int slot = 0; slot < NS; ++slot)
                G[slot >> 2][slot & 3] = bad ? 0.0 : (0.0 - bx[slot]) / s2p + G[slot >> 2][slot & 3];
        }
        lpp = acc;                                                          // MALA.jl:101
    }
    WS_WG2(3);
    (void)oos;
    double qb = 0.0;
#pragma unroll
    for (int slot = 0; slot < NS; ++slot) {
        const bool v = glm_valid(a, p, slot);
        const double xv = v ? xo[slot] : 0.0;
        const double e = (bx[slot] + half * G[slot >> 2][slot & 3]) - xv;           // MALA.jl:104-105
        if (v) qb = qb + ((-(e * e)) / twoh - Lc);
    }
    qb = glm_sum(a, p, GlmLds{}, qb);
    WS_WG2(4);
    const double ratio = ((lpp + qb) - lp) - qf;                   // MALA.jl:107
    const bool acc = glm_mh_short_circuit(rs, chain, (uint32_t)i, ratio);
    WS_WG2(5);
    int64_t kk;
    const bool kept = kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk);
    double* const ks = kept && s.samples ? s.samples + (size_t)kk * (size_t)s.d * (size_t)s.C : nullptr;
    double* const kg = kept && s.grads ? s.grads + (size_t)kk * (size_t)s.d * (size_t)s.C : nullptr;
    if (p.live) {
        // an accepted proposal is the new state; a rejected one leaves the state in HBM as it is.  Kept steps (one in
        // `thinning`, wave-uniform) write the rows, a rejected lane's gradient reloaded in groups of 8 slots with
        // every load unconditional (a masked load per slot waited for each in turn)
        double* const xw = a.st.x + (size_t)(4 * p.q) * ld + (size_t)p.c;
        double* const gw = a.st.g + (size_t)(4 * p.q) * ld + (size_t)p.c;
        const size_t Cs = (size_t)s.C;
        if (acc) {
#pragma unroll
            for (int slot = 0; slot < NS; ++slot) {
                if (!glm_valid(a, p, slot)) continue;
                const size_t r = (size_t)(16 * (slot >> 2) + (slot & 3));
                xw[r * ld] = bx[slot];
                gw[r * ld] = G[slot >> 2][slot & 3];
            }
        }
        if (ks || kg) {
#pragma unroll
            for (int slot = 0; slot < NS; ++slot) {
                if (!glm_valid(a, p, slot)) continue;
                const size_t r = (size_t)(16 * (slot >> 2) + (slot & 3));
                const size_t ko = (size_t)(4 * p.q + r) * Cs + (size_t)p.c;
                if (ks) ks[ko] = acc ? bx[slot] : xo[slot];
                if (kg) kg[ko] = acc ? G[slot >> 2][slot & 3] : *(gdouble*)(gl + r * ld);
            }
        }
    }
    WS_WG2(6);
    double hn = h;
    if (acc) {
        lp = lpp;
        if (sa.tuner) n_acc += 1;
    }
    if (kept) glm_store_bit(a, p, kk, acc);
    if (sa.tuner && i <= s.tuner_burnin && (i % sa.adapt_step) == 0) {   // MALA.jl:116-118
        hn = h * glm_tune_factor(n_acc, n_prop, sa.target_rate);
        n_acc = 0;
        n_prop = 0;
    }
    if (p.live && p.q == 0) {
        a.st.lp[p.c] = lp;
        if (sa.tuner) {
            a.st.t_step[p.c] = hn;
            a.st.t_acc[p.c] = n_acc;
            a.st.t_prop[p.c] = n_prop;
        }
    }
    glm_count_evals(a, p, s.nsteps);
    WS_WG(6);
}

// storeLeaps: leap l's state into the record, [l][d][C] and [l][C] (HMC.jl:145-150)
template <int NM>
__device__ __forceinline__ void glm_rec_put(const GlmArgs& a, const GlmPos& p, int64_t l, const double (&x)[4 * NM],
                                            const f64x4 (&g)[NM], const double (&m)[4 * NM], double lpv, double Hv) {
    if (l > a.rec.cap) return;
    glm_store_kept<NM>(a, p, l, a.rec.pars, x);
    glm_store_kept4<NM>(a, p, l, a.rec.grads, g);
    glm_store_kept<NM>(a, p, l, a.rec.mom, m);
    if (p.live && p.q == 0 && p.slice == 0) {
        a.rec.lp[(size_t)l * (size_t)a.s.C + (size_t)p.c] = lpv;
        a.rec.H[(size_t)l * (size_t)a.s.C + (size_t)p.c] = Hv;
    }
}

// REC: record the trajectory of the launch's single step (storeLeaps) and leave the chains where they are
template <int NM, int NW, bool DA, bool REC = false>
__global__ __launch_bounds__(glm_block<NW>()) void glm_hmc(GlmArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const GlmPos p = glm_pos(a);
    const GlmLds L = glm_lds(a, smem);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    const int64_t cc = p.live ? p.c : 0;
    const bool tuned = !DA && sa.tuner;
    const int64_t max_leaps = sa.max_leaps;
    double lp = a.st.lp[cc];
    double eps = (DA || tuned) ? a.st.t_step[cc] : sa.leap_step;
    int64_t nl_fixed = tuned ? (int64_t)a.st.t_leaps[cc] : sa.n_leaps;
    double eps_bar = DA ? a.st.t_bar[cc] : 0.0;
    double h_bar = DA ? a.st.t_h[cc] : 0.0;
    int32_t n_acc = tuned ? a.st.t_acc[cc] : 0;
    int32_t n_prop = tuned ? a.st.t_prop[cc] : 0;
    const double mu = DA ? det_log(10.0) : 0.0;
    int64_t n_evals = 0;
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        if (tuned) n_prop += 1;
        double x[(4 * NM)], m[(4 * NM)];
        f64x4 g[NM];
        glm_normals<NM>(p, rs, chain, (uint32_t)i, a.s.d, m);          // state0.m = randn(model.size)
        double mm = 0.0;
#pragma unroll
        for (int slot = 0; slot < (4 * NM); ++slot)
            if (glm_valid(a, p, slot)) mm = __builtin_fma(m[slot], m[slot], mm);
        const double H0 = -lp + 0.5 * glm_sum(a, p, L, mm);         // update!(state0)
        glm_load<NM>(a, p, a.st.x, x);
        glm_load4<NM>(a, p, a.st.g, g);
        if (REC) glm_rec_put<NM>(a, p, 0, x, g, m, lp, H0);             // leapStates[1] = deepcopy(state0)
        int64_t nl;
        if (DA) {
            const double r = round_away(sa.len / eps);              // HMCDA.jl:104
            nl = r < 1.0 ? 1 : (r > (double)max_leaps ? max_leaps : (int64_t)r);
        } else {
            nl = nl_fixed;
        }
        n_evals += nl;
        // the workgroup runs its longest trajectory; a d-sliced chain tile whose chains have all finished theirs
        // stops computing (glm_eval on = false: it takes its share of the staging and the barriers, and keeps its
        // last evaluation, made at the same x), so the other tile's waves have the SIMDs to themselves
        int64_t nl_tile = nl;
        const int64_t nl_wg = (DA || tuned) ? ((GLM_TILE_SKIP && NW > 1 && NW < 8) ? glm_max_tile(L, nl, p.live, p.tile, nl_tile)
                                                                                   : glm_max(L, nl, p.live))
                                            : nl;
        if (!(GLM_TILE_SKIP && NW > 1 && NW < 8 && (DA || tuned))) nl_tile = nl_wg;
        double lpl = lp;
        for (int64_t l = 0; l < nl_wg; ++l) {
            const bool active = l < nl;                              // chains that finished keep still
            if (active) {
#pragma unroll
                for (int slot = 0; slot < (4 * NM); ++slot) {
                    m[slot] = m[slot] + (0.5 * g[slot >> 2][slot & 3]) * eps;   // n.m += 0.5*n.grad*ve
                    x[slot] = x[slot] + eps * m[slot];                          // n.pars += ve * n.m
                }
            }
            bool oos;
            // d-slices: the momentum waits in HBM while the evaluation runs (its 4 NM doubles a lane would otherwise
            // be spilled inside the tile loop at the 256-register budget); plain stores and loads, bitwise the same
            constexpr bool kPark = NW > 1 && !REC;
            if (kPark && p.live) {
                double* mp = glm_lane_ptr(p, a.st.mom, s.ld, p.c);
#pragma unroll
                for (int slot = 0; slot < (4 * NM); ++slot) mp[(size_t)(16 * (slot >> 2) + (slot & 3)) * (size_t)s.ld] = m[slot];
            }
            const bool tile_on = l < nl_tile;                                // wave-uniform
            const double lpe = glm_eval<NM, NW, true>(a, p, L, x, g, oos, tile_on);   // calc!(n, ll); same x -> same (lp, g)
            if (tile_on) lpl = lpe;
            if (kPark) {
                const double* mp = glm_lane_ptr(p, a.st.mom, s.ld, p.live ? p.c : 0);
#pragma unroll
                for (int slot = 0; slot < (4 * NM); ++slot) m[slot] = mp[(size_t)(16 * (slot >> 2) + (slot & 3)) * (size_t)s.ld];
            }
            if (active) {
#pragma unroll
                for (int slot = 0; slot < (4 * NM); ++slot) m[slot] = m[slot] + (0.5 * g[slot >> 2][slot & 3]) * eps;
            }
            if (REC) {
                double m2 = 0.0;
#pragma unroll
                for (int slot = 0; slot < (4 * NM); ++slot)
                    if (glm_valid(a, p, slot)) m2 = __builtin_fma(m[slot], m[slot], m2);
                const double Hl = -lpl + 0.5 * glm_sum(a, p, L, m2);      // update!(n): every wave reaches it
                if (active) glm_rec_put<NM>(a, p, l + 1, x, g, m, lpl, Hl);
            }
        }
        if (REC) {                                                       // uniform: every wave returns here
            if (p.live && p.q == 0 && p.slice == 0) a.rec.nl[p.c] = (int32_t)nl;
            return;
        }
        mm = 0.0;
#pragma unroll
        for (int slot = 0; slot < (4 * NM); ++slot)
            if (glm_valid(a, p, slot)) mm = __builtin_fma(m[slot], m[slot], mm);
        const double H = -lpl + 0.5 * glm_sum(a, p, L, mm);
        const u32x4 w = rs.block(chain, (uint32_t)i, 0u, TAG_ACCEPT);
        const double u = uniform52(w.x, w.y);
        double pa = 0.0;
        bool acc;
        if (DA) {
            pa = __builtin_fmin(1.0, det_exp(H0 - H));              // HMCDA.jl:120
            acc = u < pa;
        } else {
            acc = u < det_exp(H0 - H);                              // HMC.jl:154
        }
        if (acc) {
            glm_store<NM>(a, p, a.st.x, s.ld, x);
            glm_store4<NM>(a, p, a.st.g, s.ld, g);
            lp = lpl;
            if (tuned) n_acc += 1;
        }
        int64_t kk;
        if (kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk)) {
            if (!acc) {
                glm_load<NM>(a, p, a.st.x, x);
                glm_load4<NM>(a, p, a.st.g, g);
            }
            glm_store_kept<NM>(a, p, kk, s.samples, x);
            glm_store_kept4<NM>(a, p, kk, s.grads, g);
            glm_store_bit(a, p, kk, acc);
        }
        if (DA) {
            const double di = (double)i;
            if (di < (double)s.tuner_burnin) {                      // HMCDA.jl:133-138
                double eta = 1.0 / (di + sa.t0);
                h_bar = (1.0 - eta) * h_bar + eta * (sa.rate - pa);
                eps = det_exp(mu - (__builtin_sqrt(di) * h_bar) / sa.shrinkage);
                eta = det_exp(det_log(di) * (-sa.step));
                eps_bar = det_exp((1.0 - eta) * det_log(eps_bar) + eta * det_log(eps));
            } else {
                eps = eps_bar;
            }
        } else if (tuned && i <= s.tuner_burnin && (i % sa.adapt_step) == 0) {
            eps = eps * glm_tune_factor(n_acc, n_prop, sa.target_rate);
            double nlf = __builtin_ceil(sa.target_path / eps);
            if (nlf > (double)sa.max_step) nlf = (double)sa.max_step;
            if (nlf > (double)max_leaps) nlf = (double)max_leaps;
            nl_fixed = (int64_t)nlf;
            n_acc = 0;
            n_prop = 0;
        }
    }
    if (p.live && p.q == 0 && p.slice == 0) {
        a.st.lp[p.c] = lp;
        if (DA || tuned) a.st.t_step[p.c] = eps;
        if (DA) {
            a.st.t_bar[p.c] = eps_bar;
            a.st.t_h[p.c] = h_bar;
        } else if (tuned) {
            a.st.t_leaps[p.c] = (int32_t)nl_fixed;
            a.st.t_acc[p.c] = n_acc;
            a.st.t_prop[p.c] = n_prop;
        }
    }
    glm_count_evals(a, p, n_evals);
}

static GlmArgs glm_args(const KernelArgs& k, const GlmShape& g) {
    GlmArgs a;
    a.s = k.s;
    a.sa = k.sa;
    a.m = k.m;
    a.st = k.st;
    a.g = g;
    a.rec = LeapRec{};
    return a;
}

static unsigned glm_grid(int64_t C, const GlmShape& g) {
    const int64_t chains_per_wg = 16 * g.tpw;
    return (unsigned)((C + chains_per_wg - 1) / chains_per_wg);
}

}  // namespace mcmc

#ifdef GLM_MALA1_UNIT
#ifdef GLM_WS_STAMP
extern "C" int mcmc_debug_ws_stamps(unsigned* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mcmc::g_ws_stamps), sizeof(mcmc::g_ws_stamps)) == hipSuccess ? 0 : 4;
}
extern "C" int mcmc_debug_ws_wg(unsigned* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mcmc::g_ws_wg), sizeof(mcmc::g_ws_wg)) == hipSuccess ? 0 : 4;
}
extern "C" int mcmc_debug_ws_wg2(unsigned* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mcmc::g_ws_wg2), sizeof(mcmc::g_ws_wg2)) == hipSuccess ? 0 : 4;
}
#endif
// glm_mala1.hip: the single-slice MALA kernels only, in a translation unit built with machine LICM
hipError_t mcmc_launch_glm_mala1(int nm, const mcmc::GlmArgs& a, size_t lds, dim3 grid, hipStream_t st) {
    using namespace mcmc;
#if GLM_MALA1_WS
    (void)lds;
    const size_t lw = glm_ws_lds_doubles(a.g.nm) * sizeof(double);
    const bool unit = a.m.prior_sigma == 1.0;                 // the prior's divisions are exact no-ops (glm_mala1ws)
    switch (nm) {
        case 1: glm_mala1ws<1><<<grid, 512, lw, st>>>(a); break;
        case 2: glm_mala1ws<2><<<grid, 512, lw, st>>>(a); break;
        case 4: glm_mala1ws<4><<<grid, 512, lw, st>>>(a); break;
        case 8:
            if (unit) glm_mala1ws<8, true><<<grid, 512, lw, st>>>(a);
            else glm_mala1ws<8><<<grid, 512, lw, st>>>(a);
            break;
        default: return hipErrorInvalidValue;
    }
#else
    constexpr int B = glm_block<1>();
    switch (nm) {
        case 1: glm_mala1<1><<<grid, B, lds, st>>>(a); break;
        case 2: glm_mala1<2><<<grid, B, lds, st>>>(a); break;
        case 4: glm_mala1<4><<<grid, B, lds, st>>>(a); break;
        case 8: glm_mala1<8><<<grid, B, lds, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
#endif
    return hipGetLastError();
}
#else
hipError_t mcmc_launch_glm_mala1(int nm, const mcmc::GlmArgs& a, size_t lds, dim3 grid, hipStream_t st);

mcmc::GlmShape mcmc_glm_shape(int d, int64_t n) {
    // d <= 128: one wave per 16-chain tile, DS = d_pad = 16 NM (NM a power of two, pipelined glm_eval1), 4 tiles
    // per workgroup;
    // 128 < d <= 256: NW = 4 slices of DS = 64 coordinates (NM = 4), two 16-chain tiles per 8-wave workgroup;
    // 256 < d <= 512: NW = 4 slices of DS = 128 (NM = 8), two tiles per workgroup, so each staged X tile feeds 32
    // chains (round 4: config 5 0.557 -> 0.582 of the fp64 MFMA spec against 64-wide slices on one box; at d = 256
    // 128-wide slices measured 0.30 against 0.53, two waves a tile);
    // 512 < d <= 1024: NW = 8 slices of DS = 128 coordinates (NM = 8), one tile per workgroup; d_pad = 1024 keeps
    // one LDS tile buffer (glm_xbufs).
    // The slice geometry fixes each chain's summation order, so it is a function of d alone, restated by the oracle
    // (orc_glm_geometry); no run-time switch changes it.
    mcmc::GlmShape g{};
    if (d <= 128) {
        int nm = 1;
        while (16 * nm < d) nm *= 2;
        g.nw = 1;
        g.nm = nm;
    } else if (d <= 256) {
        int nw = 4;
        while (64 * nw < d) nw *= 2;
        g.nw = nw;
        g.nm = 4;
    } else {
        int nw = 2;
        while (128 * nw < d) nw *= 2;
        g.nw = nw;
        g.nm = 8;
    }
    g.ds = 16 * g.nm;
    g.d_pad = g.ds * g.nw;
    g.tpw = g.nw == 1 ? 4 : 8 / g.nw;
    g.lds_stride = mcmc::glm_row_stride(g.d_pad);
    g.ts = mcmc::glm_tile_doubles(g.d_pad);
    g.n_pad = (n + 15) / 16 * 16;
    return g;
}

int mcmc_glm_max_d() { return 1024; }

// steps one launch of the regression step kernel may fuse (0: any): the single-slice MALA kernel is a
// one-step kernel (glm_mala1)
int mcmc_glm_steps_per_launch(int d, int64_t n, int sampler_kind) {
    const mcmc::GlmShape g = mcmc_glm_shape(d, n);
    return (g.nw == 1 && sampler_kind == mcmc::SK_MALA) ? 1 : 0;
}

int mcmc_glm_d_pad(int d) { return mcmc_glm_shape(d, 1).d_pad; }

int mcmc_glm_tiles_per_wg(int d) { return mcmc_glm_shape(d, 1).tpw; }

size_t mcmc_glm_image_doubles(int d, int64_t n) {
    const mcmc::GlmShape g = mcmc_glm_shape(d, n);
    return (size_t)(g.n_pad / 16) * (size_t)g.ts;
}

// the staged-tile image of X [n][d] (row-major) and Y [n] (glm_layout.hpp): tile t = rows 16t..16t+15 at
// positions glm_pos(k) of stride S, then Y; zeros elsewhere (padded rows, coordinates k >= d, gaps)
void mcmc_glm_pack_image(int d, int64_t n, const double* X, const double* Y, const double* B, double* img) {
    const mcmc::GlmShape g = mcmc_glm_shape(d, n);
    const size_t total = mcmc_glm_image_doubles(d, n);
    for (size_t i = 0; i < total; ++i) img[i] = 0.0;
    const int S = g.lds_stride, YO = mcmc::glm_y_offset(g.d_pad), BO = mcmc::glm_b_offset(g.d_pad);
    for (int64_t i = 0; i < n; ++i) {
        double* tile = img + (size_t)(i / 16) * (size_t)g.ts;
        const int r = (int)(i % 16);
        for (int k = 0; k < d; ++k) tile[r * S + k] = X[(size_t)i * d + k];
        tile[YO + r] = Y[i];
        tile[BO + r] = B ? B[i] : 0.0;
    }
    if (B)
        for (int64_t i = n; i < g.n_pad; ++i) img[(size_t)(i / 16) * (size_t)g.ts + BO + (int)(i % 16)] = -HUGE_VAL;
}

template <int NM, int NW>
static hipError_t glm_step_nm(const mcmc::GlmArgs& a, size_t lds, dim3 grid, hipStream_t st) {
    using namespace mcmc;
    constexpr int B = glm_block<NW>();
    switch (a.sa.kind) {
        case SK_RWM: mcmc_note_step_kernel("glm_rwm<%d, %d>", NM, NW); break;
        case SK_MALA:
            if (NW == 1 && GLM_MALA1_WS && NM == 8 && a.m.prior_sigma == 1.0)
                mcmc_note_step_kernel("glm_mala1ws<%d, true>", NM);          // the unit-prior instance
            else if (NW == 1) mcmc_note_step_kernel(GLM_MALA1_WS ? "glm_mala1ws<%d>" : "glm_mala1<%d>", NM);
            else mcmc_note_step_kernel("glm_mala<%d, %d>", NM, NW);
            break;
        case SK_HMC: mcmc_note_step_kernel("glm_hmc<%d, %d, false>", NM, NW); break;
        case SK_HMCDA: mcmc_note_step_kernel("glm_hmc<%d, %d, true>", NM, NW); break;
        case SK_RAM: mcmc_note_step_kernel("glm_ram<%d, %d>", NM, NW); break;
        default: break;
    }
    switch (a.sa.kind) {
        case SK_RWM: glm_rwm<NM, NW><<<grid, B, lds, st>>>(a); break;
        case SK_MALA:
            if constexpr (NW == 1) return mcmc_launch_glm_mala1(NM, a, lds, grid, st);   // glm_mala1.hip
            else glm_mala<NM, NW><<<grid, B, lds, st>>>(a);
            break;
        case SK_HMC: glm_hmc<NM, NW, false><<<grid, B, lds, st>>>(a); break;
        case SK_HMCDA: glm_hmc<NM, NW, true><<<grid, B, lds, st>>>(a); break;
        case SK_RAM:
            if constexpr (NW == 1 && NM <= 2) {
                glm_ram<NM, NW><<<grid, B, lds, st>>>(a);
                break;
            }
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t mcmc_launch_glm_step(const mcmc::KernelArgs& k, hipStream_t st) {
    using namespace mcmc;
    const GlmShape g = mcmc_glm_shape(k.s.d, k.m.n);
    const GlmArgs a = glm_args(k, g);
    const size_t lds = glm_lds_bytes(g);
    const dim3 grid(glm_grid(k.s.C, g));
    switch (g.nm * 10 + g.nw) {
        case 11: return glm_step_nm<1, 1>(a, lds, grid, st);
        case 21: return glm_step_nm<2, 1>(a, lds, grid, st);
        case 41: return glm_step_nm<4, 1>(a, lds, grid, st);
        case 81: return glm_step_nm<8, 1>(a, lds, grid, st);
        case 44: return glm_step_nm<4, 4>(a, lds, grid, st);
        case 48: return glm_step_nm<4, 8>(a, lds, grid, st);
        case 82: return glm_step_nm<8, 2>(a, lds, grid, st);
        case 84: return glm_step_nm<8, 4>(a, lds, grid, st);
        case 88: return glm_step_nm<8, 8>(a, lds, grid, st);
        default: return hipErrorInvalidValue;
    }
}

template <int NM, int NW>
static hipError_t glm_rec_nm(const mcmc::GlmArgs& a, size_t lds, dim3 grid, hipStream_t st) {
    using namespace mcmc;
    constexpr int B = glm_block<NW>();
    if (a.sa.kind == SK_HMCDA) glm_hmc<NM, NW, true, true><<<grid, B, lds, st>>>(a);
    else glm_hmc<NM, NW, false, true><<<grid, B, lds, st>>>(a);
    return hipGetLastError();
}

hipError_t mcmc_launch_glm_record(const mcmc::KernelArgs& k, const mcmc::LeapRec& r, hipStream_t st) {
    using namespace mcmc;
    if (k.sa.kind != SK_HMC && k.sa.kind != SK_HMCDA) return hipErrorInvalidValue;
    const GlmShape g = mcmc_glm_shape(k.s.d, k.m.n);
    GlmArgs a = glm_args(k, g);
    a.rec = r;
    const size_t lds = glm_lds_bytes(g);
    const dim3 grid(glm_grid(k.s.C, g));
    switch (g.nm * 10 + g.nw) {
        case 11: return glm_rec_nm<1, 1>(a, lds, grid, st);
        case 21: return glm_rec_nm<2, 1>(a, lds, grid, st);
        case 41: return glm_rec_nm<4, 1>(a, lds, grid, st);
        case 81: return glm_rec_nm<8, 1>(a, lds, grid, st);
        case 44: return glm_rec_nm<4, 4>(a, lds, grid, st);
        case 48: return glm_rec_nm<4, 8>(a, lds, grid, st);
        case 82: return glm_rec_nm<8, 2>(a, lds, grid, st);
        case 84: return glm_rec_nm<8, 4>(a, lds, grid, st);
        case 88: return glm_rec_nm<8, 8>(a, lds, grid, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t mcmc_launch_glm_eval(const mcmc::KernelArgs& k, const double* xin, double* lp, double* g, int check,
                                hipStream_t st) {
    using namespace mcmc;
    const GlmShape gs = mcmc_glm_shape(k.s.d, k.m.n);
    const GlmArgs a = glm_args(k, gs);
    const dim3 grid(glm_grid(k.s.C, gs));
    const size_t lds = glm_lds_bytes(gs);
    switch (gs.nm * 10 + gs.nw) {
        case 11: glm_eval_kernel<1, 1><<<grid, glm_block<1>(), lds, st>>>(a, xin, lp, g, check); break;
        case 21: glm_eval_kernel<2, 1><<<grid, glm_block<1>(), lds, st>>>(a, xin, lp, g, check); break;
        case 41: glm_eval_kernel<4, 1><<<grid, glm_block<1>(), lds, st>>>(a, xin, lp, g, check); break;
        case 81: glm_eval_kernel<8, 1><<<grid, glm_block<1>(), lds, st>>>(a, xin, lp, g, check); break;
        case 44: glm_eval_kernel<4, 4><<<grid, glm_block<4>(), lds, st>>>(a, xin, lp, g, check); break;
        case 48: glm_eval_kernel<4, 8><<<grid, glm_block<8>(), lds, st>>>(a, xin, lp, g, check); break;
        case 82: glm_eval_kernel<8, 2><<<grid, glm_block<2>(), lds, st>>>(a, xin, lp, g, check); break;
        case 84: glm_eval_kernel<8, 4><<<grid, glm_block<4>(), lds, st>>>(a, xin, lp, g, check); break;
        case 88: glm_eval_kernel<8, 8><<<grid, glm_block<8>(), lds, st>>>(a, xin, lp, g, check); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
#ifdef GLM_STAMP
extern "C" int mcmc_debug_glm_stamps(long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mcmc::g_glm_stamps), sizeof(mcmc::g_glm_stamps)) == hipSuccess ? 0 : 4;
}
#endif
#endif  // GLM_MALA1_UNIT
