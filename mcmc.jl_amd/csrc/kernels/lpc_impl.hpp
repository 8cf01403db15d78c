// lpc_impl.hpp -- lane-per-chain kernels (d <= 32): one thread = one chain; see samplers.hpp for the
// step code and its reference lines.  Included by one translation unit per model (lpc_<model>.hip)
// so that the instantiations compile in parallel; lpc.hip dispatches on the model kind.
#pragma once
#include "../samplers.hpp"
#include "layout_api.hpp"

namespace mcmc {

// F: d == 4 NB (LaneChain FULL); US: uniform RWM scale
template <int NB, bool F, class M, bool US>
__global__ __launch_bounds__(kBlock, 2) void lpc_rwm(KernelArgs a) { rwm_body<LaneChain<NB, F>, M, US>(a); }
template <int NB, bool F, class M>
__global__ __launch_bounds__(kBlock, 2) void lpc_mala(KernelArgs a) { mala_body<LaneChain<NB, F>, M>(a); }
template <int NB, bool F, class M, bool DA>
__global__ __launch_bounds__(kBlock) void lpc_hmc(KernelArgs a) { hmc_body<LaneChain<NB, F>, M, DA>(a); }
template <int NB, class M>
__global__ __launch_bounds__(kBlock) void lpc_eval(KernelArgs a, const double* xin, double* lp, double* g,
                                                   int32_t check) {
    eval_body<LaneChain<NB>, M>(a, xin, lp, g, check);
}

// RWM for a handful of chains (C <= 64; config 1 is one chain), where one lane per chain leaves the chip idle
// and each step is a chain of dependent operations: the Philox / Box-Muller work and the accept draw of the
// next S = 256 / C steps of every chain are spread over the block's 256 threads (thread w: chain w % C, step
// w / C) and staged in LDS, then lane c of wave 0 runs chain c's S accept steps from there.  rwm_body's
// operations on the same values (x + RN(z scale), the short-circuit test against det_log(u)), so the chains are
// bitwise the same.
constexpr int kLaMaxChains = 64;
template <int NB, class M, bool US>
__global__ __launch_bounds__(kBlock) void lpc_rwm_la(KernelArgs a) {
    using P = LaneChain<NB, false>;
    constexpr int NC = P::NC;
    const StepArgs& s = a.s;
    const P p(s);                                    // stages the Box-Muller tables (every thread)
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const int C = (int)s.C;
    const int S = kBlock / C;
    __shared__ double dz_l[kBlock][NC];
    __shared__ double lu_l[kBlock];
    const int w = (int)threadIdx.x;
    double x[NC], sc[NC];
    p.load(a.st.x, s.ld, x);
#pragma unroll
    for (int k = 0; k < NC; ++k) sc[k] = p.valid(k) ? (US ? s.scale1 : s.scale[p.coord(k)]) : 0.0;
    double lp = p.load_scalar(a.st.lp);
    // kept steps (kept_index) tracked incrementally: i_loc = burnin + 1 + kk thinning <= len; no 64-bit division
    // on the dependent per-step path
    const int64_t iloc0 = s.step_begin - s.run_step0;
    int64_t kk_next = iloc0 > s.burnin + 1 ? (iloc0 - s.burnin - 1 + s.thinning - 1) / s.thinning : 0;
    int64_t kept_next = s.burnin + 1 + kk_next * s.thinning;
    for (int t0 = 0; t0 < s.nsteps; t0 += S) {
        const int nb = s.nsteps - t0 < S ? s.nsteps - t0 : S;
        const int sw = w / C, cw = w - sw * C;
        if (sw < nb) {                               // RNG of (chain cw, step t0 + sw)
            const uint32_t chain = s.chain0 + (uint32_t)cw;
            const uint32_t i = (uint32_t)(s.step_begin + t0 + sw);
            double z[NC];
            gen_normals(p, rs, chain, i, z);
#pragma unroll
            for (int k = 0; k < NC; ++k) dz_l[w][k] = z[k] * sc[k];           // randn(d) .* scale
            const u32x4 u = rs.block(chain, i, 0u, TAG_ACCEPT);
            lu_l[w] = det_log(uniform53(u.x, u.y));                             // log(rand())
        }
        __syncthreads();
        if (w < 64) {                                // wave 0: lane c is chain c
            for (int j = 0; j < nb; ++j) {
                const int64_t i = s.step_begin + t0 + j;
                const int item = p.live ? j * C + w : 0;
                double xp[NC];
#pragma unroll
                for (int k = 0; k < NC; ++k) xp[k] = x[k] + dz_l[item][k];     // pars + randn(d) .* scale
                bool oos;
                const double lpp = eval_lp(p, model, xp, oos);
                const double ratio = lpp - lp;
                const bool acc = ratio > 0.0 || ratio > lu_l[item];             // RWM.jl:63
                if (acc) {
#pragma unroll
                    for (int k = 0; k < NC; ++k) x[k] = xp[k];
                    lp = lpp;
                }
                const int64_t iloc = i - s.run_step0;
                if (iloc == kept_next && iloc <= s.len) {                      // SerialMC.jl:49
                    p.store_kept(s, kk_next, x, s.samples);
                    p.store_bit(s, kk_next, acc);
                    kk_next += 1;
                    kept_next += s.thinning;
                }
            }
        }
        __syncthreads();
    }
    p.store(a.st.x, s.ld, x);
    p.store_t(a.st.lp, lp);
    p.count_evals(s, s.nsteps);
}

template <int NB, bool F, class M>
static hipError_t lpc_launch_model(const KernelArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    const char* b = F ? "true" : "false";
    const char* us = a.s.scale_uniform ? "true" : "false";
    switch (a.sa.kind) {
        case SK_RWM:
            if (a.s.C <= kLaMaxChains) {
                mcmc_note_step_kernel("lpc_rwm_la<%d, %s, %s>", NB, M::kName, us);
                if (a.s.scale_uniform) lpc_rwm_la<NB, M, true><<<1, kBlock, 0, st>>>(a);
                else lpc_rwm_la<NB, M, false><<<1, kBlock, 0, st>>>(a);
                break;
            }
            mcmc_note_step_kernel("lpc_rwm<%d, %s, %s, %s>", NB, b, M::kName, us);
            if (a.s.scale_uniform) lpc_rwm<NB, F, M, true><<<grid, kBlock, 0, st>>>(a);
            else lpc_rwm<NB, F, M, false><<<grid, kBlock, 0, st>>>(a);
            break;
        case SK_MALA:
            mcmc_note_step_kernel("lpc_mala<%d, %s, %s>", NB, b, M::kName);
            lpc_mala<NB, F, M><<<grid, kBlock, 0, st>>>(a);
            break;
        case SK_HMC:
            mcmc_note_step_kernel("lpc_hmc<%d, %s, %s, false>", NB, b, M::kName);
            lpc_hmc<NB, F, M, false><<<grid, kBlock, 0, st>>>(a);
            break;
        case SK_HMCDA:
            mcmc_note_step_kernel("lpc_hmc<%d, %s, %s, true>", NB, b, M::kName);
            lpc_hmc<NB, F, M, true><<<grid, kBlock, 0, st>>>(a);
            break;
        default: return hipErrorInvalidValue;
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
    switch ((a.s.d + 3) / 4) {
        case 1: lpc_eval<1, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 2: lpc_eval<2, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 3: lpc_eval<3, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 4: lpc_eval<4, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 5: lpc_eval<5, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 6: lpc_eval<6, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 7: lpc_eval<7, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 8: lpc_eval<8, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// storeLeaps records (samplers.hpp hmc_record_body), generic mapping only: a diagnostic
template <int NB, class M, bool DA>
__global__ __launch_bounds__(kBlock) void lpc_hmc_rec(KernelArgs a, LeapRec r) { hmc_record_body<LaneChain<NB>, M, DA>(a, r); }

template <class M>
static hipError_t lpc_record_m(const KernelArgs& a, const LeapRec& r, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    const bool da = a.sa.kind == SK_HMCDA;
#define LPC_REC(NB)                                                       \
    case NB:                                                              \
        if (da) lpc_hmc_rec<NB, M, true><<<grid, kBlock, 0, st>>>(a, r);   \
        else lpc_hmc_rec<NB, M, false><<<grid, kBlock, 0, st>>>(a, r);     \
        break;
    switch ((a.s.d + 3) / 4) {
        LPC_REC(1) LPC_REC(2) LPC_REC(3) LPC_REC(4) LPC_REC(5) LPC_REC(6) LPC_REC(7) LPC_REC(8)
        default: return hipErrorInvalidValue;
    }
#undef LPC_REC
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
__global__ __launch_bounds__(kBlock, NB <= 4 ? 2 : 1) void lpc_ram(KernelArgs a) { ram_body<LaneChain<NB, false>, M>(a); }

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
