// lpc_impl.hpp -- lane-per-chain kernels (d <= 32): one thread = one chain; see samplers.hpp for the
// step code and its reference lines.  Included by one translation unit per model (lpc_<model>.hip)
// so that the instantiations compile in parallel; lpc.hip dispatches on the model kind.
#pragma once
#include "../samplers.hpp"
#include "layout_api.hpp"

namespace mcmc {

// F: d == 4 NB (LaneChain FULL); US: uniform RWM scale.  RWM (config 2, d = 3): 512-thread blocks reading the
// Box-Muller tables from LDS (56 KB a block: two blocks a CU, four waves per SIMD), so 2^20 chains are exactly four
// rounds of the 512 resident blocks (768-thread blocks, six waves per SIMD, left a 2/3-full last round: CU busy
// 0.87 of the launch, 1.47e11 against 1.63e11 chain-steps/s); MALA / HMC (256 threads, two waves per SIMD by their
// registers, so two blocks a CU) read them from LDS too
constexpr int kLpcRwmThreads = 512;
template <int NB, bool F, class M, bool US>
__global__ __launch_bounds__(kLpcRwmThreads) void lpc_rwm(KernelArgs a) {
    rwm_body<LaneChain<NB, F, false, kLpcRwmThreads, kTabLds>, M, US>(a);
}
// MALA / HMC block size: two 56 KB-LDS blocks a CU, sized so that they fill the occupancy the registers allow
// (d <= 4: 125 VGPRs, four waves per SIMD; d <= 8: ~155, three; d <= 16: ~200-240, two)
template <int NB>
constexpr int lpc_grad_threads() { return NB == 1 ? 512 : (NB == 2 ? 768 : 256); }
template <int NB, bool F, class M>
__global__ __launch_bounds__((lpc_grad_threads<NB>()), (lpc_grad_threads<NB>() / 256)) void lpc_mala(KernelArgs a) {
    mala_body<LaneChain<NB, F, false, lpc_grad_threads<NB>(), kTabLds>, M>(a);
}
template <int NB, bool F, class M, bool DA>
__global__ __launch_bounds__((lpc_grad_threads<NB>()), (lpc_grad_threads<NB>() / 256)) void lpc_hmc(KernelArgs a) {
    hmc_body<LaneChain<NB, F, false, lpc_grad_threads<NB>(), kTabLds>, M, DA>(a);
}
template <int NB, class M>
__global__ __launch_bounds__(kBlock) void lpc_eval(KernelArgs a, const double* xin, double* lp, double* g,
                                                   int32_t check) {
    eval_body<LaneChain<NB>, M>(a, xin, lp, g, check);
}

// 16 < d <= 32: two lanes per chain (samplers.hpp PairChain), NB Philox blocks per lane; four waves per SIMD
// Waves per SIMD (the launch bound) and block size: RWM holds x and the proposal, 16 coordinates each, in 128 VGPRs
// (4 waves: two 512-thread blocks of 56 KB LDS; 3 when d < 2 NC leaves per-coordinate masks live); MALA 3 (one
// 768-thread block; 2 with masks); HMC's x0, x, momentum and carried kicks need ~220 (2 waves, where the lane-per-
// chain d = 32 kernel fitted one).  The Box-Muller tables are read from LDS.  MALA's block sizes, measured (r3g, d = 32,
// 2^20 chains): 768 threads / LDS tables 0.0957 ms a step, 512 / LDS (two waves) 0.0966, 256 / global tables 0.1031.
template <int NB, bool F>
constexpr int lpp_mala_threads() { return F ? 768 : 512; }
template <int NB, bool F, class M, bool US>
__global__ __launch_bounds__(512, F && US ? 4 : 3) void lpp_rwm(KernelArgs a) {
    rwm_body<PairChain<NB, F, 512, kTabLds>, M, US>(a);
}
template <int NB, bool F, class M>
__global__ __launch_bounds__((lpp_mala_threads<NB, F>()), F ? 3 : 2) void lpp_mala(KernelArgs a) {
    mala_body<PairChain<NB, F, lpp_mala_threads<NB, F>(), kTabLds>, M>(a);
}
template <int NB, bool F, class M, bool DA>
__global__ __launch_bounds__(512, 2) void lpp_hmc(KernelArgs a) { hmc_body<PairChain<NB, F, 512, kTabLds>, M, DA>(a); }
template <int NB, class M>
__global__ __launch_bounds__(kBlock) void lpp_eval(KernelArgs a, const double* xin, double* lp, double* g,
                                                   int32_t check) {
    eval_body<PairChain<NB, false, kBlock, kTabGlobal>, M>(a, xin, lp, g, check);
}

// RWM for a handful of chains (C <= 64; config 1 is one chain), where one lane per chain leaves the chip idle
// and each step is a chain of dependent operations.  Wave 0's lane c runs chain c's accept chain; waves 1-3
// (192 threads: thread g draws chain g % C, step g / C) produce the Philox / Box-Muller work and the accept
// draw of the next S = 192 / C steps into the other half of a double-buffered LDS stage while wave 0 consumes
// the current half, so the generation is off the dependent path.  Wave 0 prefetches step j+1's increments into
// registers before it runs step j.  rwm_body's operations on the same values (x + RN(z scale), the
// short-circuit test against det_log(u)), so the chains are bitwise the same.
constexpr int kLaMaxChains = 64;
constexpr int kLaGen = kBlock - 64;                  // generating threads
template <int NB, class M, bool US>
__global__ __launch_bounds__(kBlock) void lpc_rwm_la(KernelArgs a) {
    using P = LaneChain<NB, false, (NB > 4)>;        // d > 16: PairChain's summation order (lpp_rwm's chains)
    constexpr int NC = P::NC;
    const StepArgs& s = a.s;
    const P p(s);                                    // stages the Box-Muller tables (every thread)
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const int C = (int)s.C;
    const int S = kLaGen / C;
    __shared__ double dz_l[2][kLaGen][NC];
    __shared__ double lu_l[2][kLaGen];
    const int w = (int)threadIdx.x;
    double sc[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) sc[k] = p.valid(k) ? (US ? s.scale1 : s.scale[p.coord(k)]) : 0.0;
    // waves 1-3: the increments randn(d) .* scale and log(rand()) of steps t0 .. t0 + S - 1 into half `buf`
    auto generate = [&](int t0, int buf) {
        const int g = w - 64;
        const int sw = g / C, cw = g - sw * C;
        if (sw < S && t0 + sw < s.nsteps) {
            const uint32_t chain = s.chain0 + (uint32_t)cw;
            const uint32_t i = (uint32_t)(s.step_begin + t0 + sw);
            double z[NC];
            gen_normals(p, rs, chain, i, z);
#pragma unroll
            for (int k = 0; k < NC; ++k) dz_l[buf][g][k] = z[k] * sc[k];               // randn(d) .* scale
            const u32x4 u = rs.block(chain, i, 0u, TAG_ACCEPT);
            lu_l[buf][g] = det_log(uniform52(u.x, u.y));                               // log(rand())
        }
    };
    double x[NC];
    double lp = 0.0;
    if (w < 64) {
        p.load(a.st.x, s.ld, x);
        lp = p.load_scalar(a.st.lp);
    } else {
        generate(0, 0);
    }
    __syncthreads();
    // kept steps (kept_index) tracked incrementally: i_loc = burnin + 1 + kk thinning <= len; no 64-bit division
    // on the dependent per-step path
    const int64_t iloc0 = s.step_begin - s.run_step0;
    int64_t kk_next = iloc0 > s.burnin + 1 ? (iloc0 - s.burnin - 1 + s.thinning - 1) / s.thinning : 0;
    int64_t kept_next = s.burnin + 1 + kk_next * s.thinning;
    const int item0 = p.live ? w : 0;               // lanes past the last chain replay chain 0 (nothing stored)
    for (int r = 0, t0 = 0; t0 < s.nsteps; ++r, t0 += S) {
        const int buf = r & 1;
        if (w >= 64) {
            if (t0 + S < s.nsteps) generate(t0 + S, buf ^ 1);
        } else {
            const int nb = s.nsteps - t0 < S ? s.nsteps - t0 : S;
            double nz[NC], nl;
#pragma unroll
            for (int k = 0; k < NC; ++k) nz[k] = dz_l[buf][item0][k];
            nl = lu_l[buf][item0];
            for (int j = 0; j < nb; ++j) {
                double dz[NC];
#pragma unroll
                for (int k = 0; k < NC; ++k) dz[k] = nz[k];
                const double lu = nl;
                if (j + 1 < nb) {                            // step j+1's increments, in flight during step j
                    const int it = (j + 1) * C + item0;
#pragma unroll
                    for (int k = 0; k < NC; ++k) nz[k] = dz_l[buf][it][k];
                    nl = lu_l[buf][it];
                }
                double xp[NC];
#pragma unroll
                for (int k = 0; k < NC; ++k) xp[k] = x[k] + dz[k];                     // pars + randn(d) .* scale
                bool oos;
                const double lpp = eval_lp(p, model, xp, oos);
                const double ratio = lpp - lp;
                const bool acc = ratio > 0.0 || ratio > lu;                            // RWM.jl:63
                if (acc) {
#pragma unroll
                    for (int k = 0; k < NC; ++k) x[k] = xp[k];
                    lp = lpp;
                }
                const int64_t iloc = s.step_begin + t0 + j - s.run_step0;
                if (iloc == kept_next && iloc <= s.len) {                            // SerialMC.jl:49
                    p.store_kept(s, kk_next, x, s.samples);
                    p.store_bit(s, kk_next, acc);
                    kk_next += 1;
                    kept_next += s.thinning;
                }
            }
        }
        __syncthreads();
    }
    if (w < 64) {
        p.store(a.st.x, s.ld, x);
        p.store_t(a.st.lp, lp);
        p.count_evals(s, s.nsteps);
    }
}

// RWM for one chain of d = D <= 4 (config 1: d = 3): path speculation.  The next 6 steps of the chain have 64
// possible accept patterns; lane b of wave 0 assumes pattern b, so its states along those steps are known in
// advance (x advances by its increment exactly at the steps b accepts) and it evaluates all 6 proposals without
// waiting for any accept test -- six independent evaluations instead of a dependent chain.  A lane is
// consistent when every accept test it computes agrees with its pattern; exactly one lane is (every lane agrees
// with the true path up to its first difference from it, where the true test contradicts it), and its states
// are the chain's: one ballot per 6 steps, and the winning lane index IS the accept pattern, so the new state is
// read with v_readlane (no LDS round trip).  The arithmetic of every state, proposal and test is rwm_body's
// (x + RN(z scale), the short-circuit test against det_log(u)) on the same values in the same order, so the chain
// is bitwise the same.  D is exact (no per-coordinate validity masks).  Waves 1-3 produce the increments and
// accept draws into a double-buffered LDS stage (as lpc_rwm_la), and copy the kept rows, staged in LDS by the
// winning lane, out as contiguous runs during the next stage half.
constexpr int kSpecK = 6;
__device__ __forceinline__ double readlane_f64(double v, int lane) {   // lane: wave-uniform
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <int D, class M, bool US>
__global__ __launch_bounds__(kBlock) void lpc_rwm_spec(KernelArgs a) {
    using P = LaneChain<1, false>;                   // RNG blocks of 4 normals: D <= 4 takes one
    constexpr int NC = P::NC;
    static_assert(D >= 1 && D <= NC, "one Philox block of normals per step");
    const StepArgs& s = a.s;
    const P p(s);                                    // stages the Box-Muller tables (every thread)
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    constexpr int S = kLaGen / kSpecK * kSpecK;      // steps per stage half: whole 6-step blocks
    __shared__ double dz_l[2][kLaGen][D];
    __shared__ double lu_l[2][kLaGen];
    __shared__ double kept_l[2][kLaGen * D];         // kept rows of a half ([row][d]), rows kinfo_l[.][0] ..
    __shared__ uint64_t kbits_l[2][kLaGen];          // and their accept words
    __shared__ int64_t kinfo_l[2][2];                // first kept row, row count
    const int w = (int)threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(w >> 6);   // wave-uniform role tests: scalar branches
    double sc[D];
#pragma unroll
    for (int k = 0; k < D; ++k) sc[k] = US ? s.scale1 : s.scale[k];
    auto generate = [&](int t0, int buf) {           // waves 1-3: thread g draws step t0 + g
        const int g = w - 64;
        if (g < S && t0 + g < s.nsteps) {
            const uint32_t i = (uint32_t)(s.step_begin + t0 + g);
            double z[NC];
            gen_normals(p, rs, s.chain0, i, z);
#pragma unroll
            for (int k = 0; k < D; ++k) dz_l[buf][g][k] = z[k] * sc[k];                // randn(d) .* scale
            const u32x4 u = rs.block(s.chain0, i, 0u, TAG_ACCEPT);
            lu_l[buf][g] = det_log(uniform52(u.x, u.y));                               // log(rand())
        }
    };
    auto flush = [&](int buf, int t, int nt) {       // threads t, t+nt, ... copy half buf's kept rows out
        const int64_t k0 = kinfo_l[buf][0], nr = kinfo_l[buf][1];
        if (s.samples != nullptr) {
            double* dst = s.samples + (size_t)k0 * D;
            for (int64_t e = t; e < nr * D; e += nt) dst[e] = kept_l[buf][e];
        }
        if (s.acc_bits != nullptr)
            for (int64_t e = t; e < nr; e += nt) s.acc_bits[(size_t)(k0 + e) * (size_t)s.nw] = kbits_l[buf][e];
    };
    double x[D];                                     // wave 0: the chain's state (uniform)
    double lp = 0.0;
    if (wave == 0) {
#pragma unroll
        for (int k = 0; k < D; ++k) x[k] = a.st.x[(size_t)k * (size_t)s.ld];
        lp = a.st.lp[0];
    } else {
        generate(0, 0);
    }
    __syncthreads();
    const int64_t iloc0 = s.step_begin - s.run_step0;
    int64_t kk_next = iloc0 > s.burnin + 1 ? (iloc0 - s.burnin - 1 + s.thinning - 1) / s.thinning : 0;
    int64_t kept_next = s.burnin + 1 + kk_next * s.thinning;
    const int b = w & 63;                            // wave 0: this lane's accept pattern
    int r = 0;
    for (int t0 = 0; t0 < s.nsteps; ++r, t0 += S) {
        const int buf = r & 1;
        if (wave != 0) {
            if (r > 0) flush(buf ^ 1, w - 64, kLaGen);      // the previous half's kept rows
            if (t0 + S < s.nsteps) generate(t0 + S, buf ^ 1);
        } else {
            const int nb = s.nsteps - t0 < S ? s.nsteps - t0 : S;
            const int64_t kfirst = kk_next;
            for (int j0 = 0; j0 < nb; j0 += kSpecK) {
                const int kb = nb - j0 < kSpecK ? nb - j0 : kSpecK;   // steps in this block (uniform)
                // the block's kept steps (SerialMC.jl:49): bit i of km
                uint32_t km = 0;
                {
                    const int64_t base = iloc0 + t0 + j0;            // i_loc of the block's first step
                    const int64_t end = base + kb - 1 < s.len ? base + kb - 1 : s.len;   // last keepable i_loc
                    if (kept_next <= end) {
                        if (s.thinning == 1) {                       // a contiguous run: bits first .. last
                            const int f = (int)(kept_next - base), l = (int)(end - base);
                            km = ((2u << l) - 1u) & ~((1u << f) - 1u);
                            kept_next = end + 1;
                        } else {
                            for (; kept_next <= end; kept_next += s.thinning) km |= 1u << (int)(kept_next - base);
                        }
                    }
                }
                // all 6 steps unconditionally (no branch between the LDS reads and the arithmetic): the stage rows of
                // steps past kb lie inside the stage (S is a multiple of 6) and only patterns with zero bits there can
                // be consistent, so those steps neither move xs nor decide ok
                bool ok = (b >> kb) == 0;                           // patterns past the block's end: not a path
                double xs[D], xh[kSpecK][D];
                double lps = lp;
#pragma unroll
                for (int k = 0; k < D; ++k) xs[k] = x[k];
#pragma unroll
                for (int i = 0; i < kSpecK; ++i) {
                    const int it = j0 + i;
                    const double lu = lu_l[buf][it];
                    double xp[D];
#pragma unroll
                    for (int k = 0; k < D; ++k) xp[k] = xs[k] + dz_l[buf][it][k];       // pars + randn(d) .* scale
                    bool oos;
                    double lpp;                                                        // model.eval
                    if constexpr (is_joint<M>::value) {
                        lpp = model.joint_lp(xp, oos);              // a joint target (OU): no per-coordinate sum
                    } else {
                        double acc0 = 0.0;
#pragma unroll
                        for (int k = 0; k < D; ++k) model.acc(acc0, xp[k]);
                        lpp = llacc_finish(model, acc0, oos);
                    }
                    const double ratio = lpp - lps;
                    const bool acc = (ratio > 0.0) | (ratio > lu);                       // RWM.jl:63
                    const bool bi = (b >> i) & 1;
                    ok = ok && (acc == bi || i >= kb);
#pragma unroll
                    for (int k = 0; k < D; ++k) xs[k] = bi ? xp[k] : xs[k];
                    lps = bi ? lpp : lps;
#pragma unroll
                    for (int k = 0; k < D; ++k) xh[i][k] = xs[k];
                }
                const uint64_t okm = __ballot(ok);
                const int src = okm ? __builtin_ctzll(okm) : 0;      // the consistent lane = the accept pattern
#pragma unroll
                for (int k = 0; k < D; ++k) x[k] = readlane_f64(xs[k], src);
                lp = readlane_f64(lps, src);
                if (km && b == src) {                                // the consistent lane stages the kept rows
                    int kr = (int)(kk_next - kfirst);
#pragma unroll
                    for (int i = 0; i < kSpecK; ++i) {
                        if ((km >> i) & 1u) {
#pragma unroll
                            for (int k = 0; k < D; ++k) kept_l[buf][kr * D + k] = xh[i][k];
                            kbits_l[buf][kr] = (uint64_t)((src >> i) & 1);
                            kr += 1;
                        }
                    }
                }
                kk_next += __builtin_popcount(km);
            }
            if (w == 0) {
                kinfo_l[buf][0] = kfirst;
                kinfo_l[buf][1] = kk_next - kfirst;
            }
        }
        __syncthreads();
    }
    if (r > 0) flush((r - 1) & 1, w, kBlock);            // the last half, by the whole block
    if (w == 0) {
#pragma unroll
        for (int k = 0; k < D; ++k) a.st.x[(size_t)k * (size_t)s.ld] = x[k];
        a.st.lp[0] = lp;
        if (s.n_evals != nullptr) atomicAdd(s.n_evals, (unsigned long long)s.nsteps);
    }
}

template <int D, class M>
static void lpc_spec_launch(const KernelArgs& a, hipStream_t st) {
    if (a.s.scale_uniform) lpc_rwm_spec<D, M, true><<<1, kBlock, 0, st>>>(a);
    else lpc_rwm_spec<D, M, false><<<1, kBlock, 0, st>>>(a);
}

// 16 < d <= 32 (NB = ceil(d/4) > 4): the two-lanes-per-chain kernels, NBL = ceil(NB / 2) blocks per lane
template <int NBL, bool F, class M>
static hipError_t lpp_launch(const KernelArgs& a, hipStream_t st) {
    auto grid = [&](int threads) { return dim3((unsigned)((a.s.C + threads / 2 - 1) / (threads / 2))); };
    const char* b = F ? "true" : "false";
    const char* us = a.s.scale_uniform ? "true" : "false";
    constexpr int TM = lpp_mala_threads<NBL, F>();
    switch (a.sa.kind) {
        case SK_RWM:
            mcmc_note_step_kernel("lpp_rwm<%d, %s, %s, %s>", NBL, b, M::kName, us);
            if (a.s.scale_uniform) lpp_rwm<NBL, F, M, true><<<grid(512), 512, 0, st>>>(a);
            else lpp_rwm<NBL, F, M, false><<<grid(512), 512, 0, st>>>(a);
            break;
        case SK_MALA:
            mcmc_note_step_kernel("lpp_mala<%d, %s, %s>", NBL, b, M::kName);
            lpp_mala<NBL, F, M><<<grid(TM), TM, 0, st>>>(a);
            break;
        case SK_HMC:
            mcmc_note_step_kernel("lpp_hmc<%d, %s, %s, false>", NBL, b, M::kName);
            lpp_hmc<NBL, F, M, false><<<grid(512), 512, 0, st>>>(a);
            break;
        case SK_HMCDA:
            mcmc_note_step_kernel("lpp_hmc<%d, %s, %s, true>", NBL, b, M::kName);
            lpp_hmc<NBL, F, M, true><<<grid(512), 512, 0, st>>>(a);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int NB, bool F, class M>
static hipError_t lpc_launch_model(const KernelArgs& a, hipStream_t st) {
    const char* us = a.s.scale_uniform ? "true" : "false";
    const bool few = a.sa.kind == SK_RWM && a.s.C <= kLaMaxChains;      // lpc_rwm_la (split order for d > 16)
    if constexpr (NB > 4) {
        if (!few) return lpp_launch<(NB + 1) / 2, F && (NB % 2 == 0), M>(a, st);
        mcmc_note_step_kernel("lpc_rwm_la<%d, %s, %s>", NB, M::kName, us);
        if (a.s.scale_uniform) lpc_rwm_la<NB, M, true><<<1, kBlock, 0, st>>>(a);
        else lpc_rwm_la<NB, M, false><<<1, kBlock, 0, st>>>(a);
    } else {
        const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
        auto gridT = [&](int threads) { return dim3((unsigned)((a.s.C + threads - 1) / threads)); };
        const char* b = F ? "true" : "false";
        switch (a.sa.kind) {
            case SK_RWM:
                if (NB == 1 && a.s.C == 1) {
                    mcmc_note_step_kernel("lpc_rwm_spec<%d, %s, %s>", (int)a.s.d, M::kName, us);
                    switch (a.s.d) {
                        case 1: lpc_spec_launch<1, M>(a, st); break;
                        case 2: lpc_spec_launch<2, M>(a, st); break;
                        case 3: lpc_spec_launch<3, M>(a, st); break;
                        default: lpc_spec_launch<4, M>(a, st); break;
                    }
                    break;
                }
                if (a.s.C <= kLaMaxChains) {
                    mcmc_note_step_kernel("lpc_rwm_la<%d, %s, %s>", NB, M::kName, us);
                    if (a.s.scale_uniform) lpc_rwm_la<NB, M, true><<<1, kBlock, 0, st>>>(a);
                    else lpc_rwm_la<NB, M, false><<<1, kBlock, 0, st>>>(a);
                    break;
                }
                mcmc_note_step_kernel("lpc_rwm<%d, %s, %s, %s>", NB, b, M::kName, us);
                {
                    const dim3 g768((unsigned)((a.s.C + kLpcRwmThreads - 1) / kLpcRwmThreads));
                    if (a.s.scale_uniform) lpc_rwm<NB, F, M, true><<<g768, kLpcRwmThreads, 0, st>>>(a);
                    else lpc_rwm<NB, F, M, false><<<g768, kLpcRwmThreads, 0, st>>>(a);
                }
                break;
            case SK_MALA:
                mcmc_note_step_kernel("lpc_mala<%d, %s, %s>", NB, b, M::kName);
                lpc_mala<NB, F, M><<<gridT(lpc_grad_threads<NB>()), lpc_grad_threads<NB>(), 0, st>>>(a);
                break;
            case SK_HMC:
                mcmc_note_step_kernel("lpc_hmc<%d, %s, %s, false>", NB, b, M::kName);
                lpc_hmc<NB, F, M, false><<<gridT(lpc_grad_threads<NB>()), lpc_grad_threads<NB>(), 0, st>>>(a);
                break;
            case SK_HMCDA:
                mcmc_note_step_kernel("lpc_hmc<%d, %s, %s, true>", NB, b, M::kName);
                lpc_hmc<NB, F, M, true><<<gridT(lpc_grad_threads<NB>()), lpc_grad_threads<NB>(), 0, st>>>(a);
                break;
            default: return hipErrorInvalidValue;
        }
    }
    return hipGetLastError();
}

// SPEC: instantiate the FULL (d == 4 NB) variants too -- for the models the benchmarks run
template <int NB, class M, bool SPEC>
static hipError_t lpc_launch_nb(const KernelArgs& a, hipStream_t st) {
    if (SPEC && a.s.d == 4 * NB) return lpc_launch_model<NB, SPEC, M>(a, st);
    return lpc_launch_model<NB, false, M>(a, st);
}

template <class M, bool SPEC>
static hipError_t lpc_step(const KernelArgs& a, hipStream_t st) {
    switch ((a.s.d + 3) / 4) {
        case 1: return lpc_launch_nb<1, M, SPEC>(a, st);
        case 2: return lpc_launch_nb<2, M, SPEC>(a, st);
        case 3: return lpc_launch_nb<3, M, SPEC>(a, st);
        case 4: return lpc_launch_nb<4, M, SPEC>(a, st);
        case 5: return lpc_launch_nb<5, M, SPEC>(a, st);
        case 6: return lpc_launch_nb<6, M, SPEC>(a, st);
        case 7: return lpc_launch_nb<7, M, SPEC>(a, st);
        case 8: return lpc_launch_nb<8, M, SPEC>(a, st);
        default: return hipErrorInvalidValue;
    }
}

template <class M>
static hipError_t lpc_eval_m(const KernelArgs& a, const double* xin, double* lp, double* g, int check,
                             hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    const dim3 grid2((unsigned)((a.s.C + kBlock / 2 - 1) / (kBlock / 2)));       // PairChain: 128 chains a block
    switch ((a.s.d + 3) / 4) {
        case 1: lpc_eval<1, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 2: lpc_eval<2, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 3: lpc_eval<3, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 4: lpc_eval<4, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 5:
        case 6: lpp_eval<3, M><<<grid2, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 7:
        case 8: lpp_eval<4, M><<<grid2, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// storeLeaps records (samplers.hpp hmc_record_body), generic mapping only: a diagnostic
template <int NB, class M, bool DA>
__global__ __launch_bounds__(kBlock) void lpc_hmc_rec(KernelArgs a, LeapRec r) { hmc_record_body<LaneChain<NB>, M, DA>(a, r); }

template <int NB, class M, bool DA>
__global__ __launch_bounds__(kBlock) void lpp_hmc_rec(KernelArgs a, LeapRec r) {
    hmc_record_body<PairChain<NB, false, kBlock, kTabGlobal>, M, DA>(a, r);
}

template <class M>
static hipError_t lpc_record_m(const KernelArgs& a, const LeapRec& r, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    const dim3 grid2((unsigned)((a.s.C + kBlock / 2 - 1) / (kBlock / 2)));
    const bool da = a.sa.kind == SK_HMCDA;
#define LPC_REC(NB)                                                       \
    case NB:                                                              \
        if (da) lpc_hmc_rec<NB, M, true><<<grid, kBlock, 0, st>>>(a, r);   \
        else lpc_hmc_rec<NB, M, false><<<grid, kBlock, 0, st>>>(a, r);     \
        break;
#define LPP_REC(NB, NBL)                                                    \
    case NB:                                                                \
        if (da) lpp_hmc_rec<NBL, M, true><<<grid2, kBlock, 0, st>>>(a, r);   \
        else lpp_hmc_rec<NBL, M, false><<<grid2, kBlock, 0, st>>>(a, r);     \
        break;
    switch ((a.s.d + 3) / 4) {
        LPC_REC(1) LPC_REC(2) LPC_REC(3) LPC_REC(4) LPP_REC(5, 3) LPP_REC(6, 3) LPP_REC(7, 4) LPP_REC(8, 4)
        default: return hipErrorInvalidValue;
    }
#undef LPC_REC
#undef LPP_REC
    return hipGetLastError();
}

}  // namespace mcmc

// one translation unit per model: LPC_UNIT(iso, IsoDot, true) defines mcmc_lpc_step_iso / mcmc_lpc_eval_iso
#define LPC_UNIT(name, Model, SPEC)                                                                      \
    hipError_t mcmc_lpc_step_##name(const mcmc::KernelArgs& a, hipStream_t st) {                         \
        return mcmc::lpc_step<mcmc::Model, SPEC>(a, st);                                                \
    }                                                                                                    \
    hipError_t mcmc_lpc_eval_##name(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, \
                                    int check, hipStream_t st) {                                         \
        return mcmc::lpc_eval_m<mcmc::Model>(a, xin, lp, g, check, st);                                 \
    }                                                                                                    \
    hipError_t mcmc_lpc_record_##name(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st) { \
        return mcmc::lpc_record_m<mcmc::Model>(a, r, st);                                               \
    }

// RAM kernels live in their own translation units (lpc_ram_*.hip, built without machine LICM: hoisted
// fp64 constants would pin the scalar file the factor addressing needs); LPC_RAM_UNIT(iso, IsoDot)
// defines mcmc_lpc_ram_iso.
namespace mcmc {
template <int NB, class M>
// d > 16: the log-target in PairChain's order (LaneChain SPLIT), as the chains' model.eval (lpp_eval) forms it.
// The next step's rvec from LDS (ram_body kZLds) and the Box-Muller tables from LDS too, except at 12 < d <= 16,
// where 56 KB of tables beside the 32 KB rvec would leave one block a CU and the registers allow two
__global__ __launch_bounds__(kBlock, NB <= 4 ? 2 : 1) void lpc_ram(KernelArgs a) {
    ram_body<LaneChain<NB, false, (NB > 4), kBlock, NB == 4 ? kTabGlobal : kTabLds>, M>(a);
}

template <class M>
static hipError_t lpc_ram_step(const KernelArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    mcmc_note_step_kernel("lpc_ram<%d, %s>", (a.s.d + 3) / 4, M::kName);
    switch ((a.s.d + 3) / 4) {
        case 1: lpc_ram<1, M><<<grid, kBlock, 0, st>>>(a); break;
        case 2: lpc_ram<2, M><<<grid, kBlock, 0, st>>>(a); break;
        case 3: lpc_ram<3, M><<<grid, kBlock, 0, st>>>(a); break;
        case 4: lpc_ram<4, M><<<grid, kBlock, 0, st>>>(a); break;
        case 5: lpc_ram<5, M><<<grid, kBlock, 0, st>>>(a); break;
        case 6: lpc_ram<6, M><<<grid, kBlock, 0, st>>>(a); break;
        case 7: lpc_ram<7, M><<<grid, kBlock, 0, st>>>(a); break;
        case 8: lpc_ram<8, M><<<grid, kBlock, 0, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
}  // namespace mcmc

#define LPC_RAM_UNIT(name, Model)                                                \
    hipError_t mcmc_lpc_ram_##name(const mcmc::KernelArgs& a, hipStream_t st) { \
        return mcmc::lpc_ram_step<mcmc::Model>(a, st);                          \
    }
