// glm_ram_wave.hip -- robust adaptive Metropolis (src/samplers/RAM.jl:41-79) on the regression targets for
// 32 < d <= 1024.  The d x d jump factor of a chain is as large as the rows of X a 16-chain MFMA tile streams per
// evaluation, so the step is split across three kernels instead of fused into glm_ram's tile loop:
//   glm_ram_prop    (once per launch sequence)  rvec = randn(d), u = S rvec, |rvec|^2; xprop = x + u      (RAM.jl:58-60)
//   glm eval kernel (every step)                lpp = log-target at xprop (the regression MFMA evaluation)
//   glm_ram_update  (every step)                the MH test (RAM.jl:62-71), the factor update (RAM.jl:74-78) with
//                                               the next step's S rvec folded into it (ram_wave_update NEXT), and
//                                               the next xprop
// The factor is the wave-per-chain layout of ram_wave.hpp: for 32 < d <= 256 two chains per wave, 32 lanes each (the
// separable targets' HalfWaveChain: a column's pivot work is shared by two chains and no lane slot lies past d), for
// d > 256 one chain per wave, its rows over the 64 lanes; x stays in the regression layout [d][ld] (the eval kernel's
// input), read and written per coordinate.  u (row layout) and |rvec|^2 wait in HBM between the kernels.  Sums: the
// matvec and the update are ram_wave.hpp's, |rvec|^2 the half-wave (d <= 256) or 64-lane wave order; oracle.c restates
// both (orc_chain, RAM on a regression target with d > 32).
#include "wpc_impl.hpp"
#include "../ram_wave.hpp"

namespace mcmc {

// A wave-per-chain policy's coordinate layout (lane l of the chain's L, slot 4 g + e <-> coordinate 4 (l + L g) + e)
// over the regression state [d][ld] and the C ABI's kept layout [nkept][d][C]; B = WaveChain (L = 64) or
// HalfWaveChain (L = 32, two chains a wave)
template <class B>
struct GlmChain : B {
    using Base = B;
    using Base::c;
    using Base::coord;
    using Base::live;
    using Base::valid;
    static constexpr int NC = Base::NC;
    static constexpr int CPW = 64 / Base::L;                    // chains per wave
    int64_t ld;
    // c0: the first chain of the launch (a half of the batch on its own stream): the policy's chain index is local
    // to the launch's grid, every array is indexed by the batch's
    __device__ GlmChain(const StepArgs& s, int64_t c0) : Base(s) {
        ld = s.ld;
        c += c0;
        live = c < s.C;
    }
    __device__ __forceinline__ int64_t cc() const { return live ? c : 0; }
    // the wave's first chain (its factor block starts the buffer resource) and this lane's byte offset in it
    __device__ __forceinline__ int64_t wave_chain0() const { return c - (int64_t)((threadIdx.x & 63) / Base::L); }
    __device__ __forceinline__ uint32_t vo(int64_t ram_ld) const {
        return (uint32_t)((threadIdx.x & 63) / Base::L) * (uint32_t)(ram_ld * 8) + (uint32_t)Base::lane * 8u;
    }
    __device__ __forceinline__ void load_glm(const double* x, double (&v)[NC]) const {
        const int64_t c0 = cc();
#pragma unroll
        for (int k = 0; k < NC; ++k) v[k] = valid(k) ? x[(size_t)coord(k) * (size_t)ld + (size_t)c0] : 0.0;
    }
    __device__ __forceinline__ void store_glm(double* x, const double (&v)[NC]) const {
        if (!live) return;
#pragma unroll
        for (int k = 0; k < NC; ++k)
            if (valid(k)) x[(size_t)coord(k) * (size_t)ld + (size_t)c] = v[k];
    }
    __device__ __forceinline__ void store_kept_glm(const StepArgs& s, int64_t kk, const double (&v)[NC]) const {
        if (s.samples == nullptr || !live) return;
        double* p = s.samples + (size_t)kk * (size_t)s.d * (size_t)s.C + (size_t)c;
#pragma unroll
        for (int k = 0; k < NC; ++k)
            if (valid(k)) p[(size_t)coord(k) * (size_t)s.C] = v[k];
    }
};
template <int G>
using GlmWaveChain = GlmChain<WaveChain<G, false, 1, kTabGlobal>>;
template <int G>
using GlmHalfWaveChain = GlmChain<HalfWaveChain<G>>;

// the per-chain buffers between the kernels: u = S rvec in row layout [C][ustride] and |rvec|^2 [C]
struct GlmRamBufs {
    double* u;
    double* nz;
    double* xprop;      // [d][ld]
    const double* lpp;  // [C]
    int64_t ustride;    // doubles of u per chain (mcmc_glm_ram_wave_ustride)
    int64_t c0;         // the launch's first chain (0, or the second half's on the second stream)
};

// the wave's chains exist (a tail wave with none leaves; with two chains a wave one half may be past C: its loads
// read chain 0 or its own allocated factor block, its stores are skipped)
template <class P>
__device__ __forceinline__ bool glm_ram_wave_live(const P& p, const StepArgs& s) {
    return p.wave_chain0() < s.C;
}

// rvec of step i, |rvec|^2 (the chain's lane order), u = S_(i-1) rvec; xprop = x + u
template <class P>
__global__ __launch_bounds__(kBlock) void glm_ram_prop(KernelArgs a, GlmRamBufs b) {
    constexpr int NC = P::NC, L = P::L, CPW = P::CPW;
    const StepArgs& s = a.s;
    const P p(s, b.c0);
    if (!glm_ram_wave_live(p, s)) return;                        // wave-uniform
    __shared__ double xpose[kBlock / 64][64 * NC];
    double* const slice = &xpose[threadIdx.x >> 6][((threadIdx.x & 63) / L) * L * NC];
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    const int d = s.d;
    const int64_t i = s.step_begin;
    double z[NC], zr[NC], u[NC], uq[NC], x[NC];
    gen_normals(p, rs, chain, (uint32_t)i, z);                    // rvec = randn(d)
    double a2 = 0.0;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        if (!p.valid(k)) z[k] = 0.0;
        a2 = __builtin_fma(z[k], z[k], a2);                       // dot(rvec, rvec)
    }
    const double nz = p.reduce(a2);
    ram_to_rows<NC, L>(slice, p.lane, z, zr);
    const int64_t ld = a.st.ram_ld;
    double* const B0 = a.st.ram_L + (uint64_t)p.wave_chain0() * (uint64_t)ld;
    const ram_rsrc_t Ss = ram_chain_rsrc(B0 + (uint64_t)((i - 1) & 1) * (uint64_t)a.st.ram_hs, ld * 8 * CPW);
    ram_wave_matvec<NC, L>(Ss, p.vo(ld), p.lane, d, zr, u);       // S * rvec
    if (p.live) {
#pragma unroll
        for (int sl = 0; sl < NC; ++sl) b.u[(size_t)p.c * (size_t)b.ustride + (size_t)(p.lane + L * sl)] = u[sl];
        if (p.lane == 0) b.nz[p.c] = nz;
    }
    ram_to_quads<NC, L>(slice, p.lane, u, uq);
    p.load_glm(a.st.x, x);
#pragma unroll
    for (int k = 0; k < NC; ++k) x[k] = x[k] + uq[k];             // RAM.jl:60
    p.store_glm(b.xprop, x);
}

// step i: accept (RAM.jl:62-71), kept rows, the factor update (RAM.jl:74-78); NEXT: step i + 1's u, |rvec|^2, xprop
template <class P, bool NEXT>
__global__ __launch_bounds__(kBlock) void glm_ram_update(KernelArgs a, GlmRamBufs b) {
    constexpr int NC = P::NC, L = P::L, CPW = P::CPW;
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const P p(s, b.c0);
    if (!glm_ram_wave_live(p, s)) return;                        // wave-uniform
    __shared__ double xpose[kBlock / 64][64 * NC];
    double* const slice = &xpose[threadIdx.x >> 6][((threadIdx.x & 63) / L) * L * NC];
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    const int d = s.d;
    const int64_t i = s.step_begin;
    double x[NC], u[NC], uq[NC];
    p.load_glm(a.st.x, x);
    const int64_t c0 = p.cc();
    double lp = a.st.lp[c0];
    const double lpp = b.lpp[c0];
#pragma unroll
    for (int sl = 0; sl < NC; ++sl) u[sl] = b.u[(size_t)c0 * (size_t)b.ustride + (size_t)(p.lane + L * sl)];
    const double nz = b.nz[c0];
    ram_to_quads<NC, L>(slice, p.lane, u, uq);
    const double ratio = lpp - lp;
    const bool acc = mh_accept_short_circuit(rs, chain, (uint32_t)i, ratio);
    if (acc) {
#pragma unroll
        for (int k = 0; k < NC; ++k) x[k] = x[k] + uq[k];         // the proposal xprop, the same sums
        lp = lpp;
    }
    Keeper keep(s);
    int64_t kk;
    if (keep.take(i, &kk)) {
        p.store_kept_glm(s, kk, x);
        p.store_bit(s, kk, acc);
    }
    const double alpha = ram_alpha(i, d, ratio, sa.rate);
    const int64_t ld = a.st.ram_ld;
    double* const B0 = a.st.ram_L + (uint64_t)p.wave_chain0() * (uint64_t)ld;
    const uint64_t hs = (uint64_t)a.st.ram_hs;
    const ram_rsrc_t Ss = ram_chain_rsrc(B0 + (uint64_t)((i - 1) & 1) * hs, ld * 8 * CPW);
    const ram_rsrc_t Sd = ram_chain_rsrc(B0 + (uint64_t)(i & 1) * hs, ld * 8 * CPW);
    double zn[NC], znr[NC], un[NC];
    double a2 = 0.0;
    if (NEXT) {
        gen_normals(p, rs, chain, (uint32_t)(i + 1), zn);          // step i + 1's rvec
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (!p.valid(k)) zn[k] = 0.0;
            a2 = __builtin_fma(zn[k], zn[k], a2);
        }
        ram_to_rows<NC, L>(slice, p.lane, zn, znr);
    }
    ram_wave_update<NC, L, NEXT>(Ss, Sd, p.vo(ld), p.lane, d, alpha, nz, u, znr, un);
    p.store_glm(a.st.x, x);
    if (p.live && p.lane == 0) a.st.lp[p.c] = lp;
    if (NEXT) {
        if (p.live) {
#pragma unroll
            for (int sl = 0; sl < NC; ++sl) b.u[(size_t)p.c * (size_t)b.ustride + (size_t)(p.lane + L * sl)] = un[sl];
        }
        const double nzn = p.reduce(a2);
        if (p.live && p.lane == 0) b.nz[p.c] = nzn;
        ram_to_quads<NC, L>(slice, p.lane, un, uq);
#pragma unroll
        for (int k = 0; k < NC; ++k) x[k] = x[k] + uq[k];
        p.store_glm(b.xprop, x);
    }
}

// batches of at least this many chains run as two halves on two streams (the eval kernel of one half beside the
// factor update of the other: MFMA and HBM); each half still fills the GPU
constexpr int64_t kRamTwoStreamMin = 8192;

template <class P>
static hipError_t glm_ram_wave_g(const KernelArgs& a0, const GlmRamBufs& b0, double* lpp, hipStream_t st,
                                 hipStream_t st2, hipEvent_t ev_fork, hipEvent_t ev_join) {
    const int64_t cpb = (int64_t)kChainsPerBlock * P::CPW;     // chains per 256-thread block
    const int64_t C = a0.s.C;
    const bool two = st2 != nullptr && C >= kRamTwoStreamMin;
    const int64_t c1 = two ? (C / 2 + 63) / 64 * 64 : C;      // 64-aligned: whole accept words and eval tiles
    struct Half {
        int64_t first, count;
        hipStream_t st;
    };
    const Half H[2] = {{0, c1, st}, {c1, C - c1, st2}};
    const int nh = two ? 2 : 1;
    hipError_t e = hipSuccess;
    if (two) {
        e = hipEventRecord(ev_fork, st);
        if (e == hipSuccess) e = hipStreamWaitEvent(st2, ev_fork, 0);
        if (e != hipSuccess) return e;
    }
    KernelArgs a = a0;
    a.s.nsteps = 1;
    GlmRamBufs b = b0;
    b.lpp = lpp;
    for (int h = 0; h < nh && e == hipSuccess; ++h) {
        b.c0 = H[h].first;
        glm_ram_prop<P><<<(unsigned)((H[h].count + cpb - 1) / cpb), kBlock, 0, H[h].st>>>(a, b);
        e = hipGetLastError();
    }
    for (int t = 0; t < a0.s.nsteps && e == hipSuccess; ++t) {
        a.s.step_begin = a0.s.step_begin + t;
        for (int h = 0; h < nh && e == hipSuccess; ++h) {
            KernelArgs ae = a;                                 // the half's chains for the eval kernel
            ae.s.C = H[h].count;
            ae.s.order = nullptr;                              // identity (no trajectory order for RAM)
            e = mcmc_launch_glm_eval(ae, b.xprop + H[h].first, lpp + H[h].first, nullptr, 0, H[h].st);
            if (e != hipSuccess) break;
            b.c0 = H[h].first;
            const dim3 grid((unsigned)((H[h].count + cpb - 1) / cpb));
            if (t + 1 < a0.s.nsteps) glm_ram_update<P, true><<<grid, kBlock, 0, H[h].st>>>(a, b);
            else glm_ram_update<P, false><<<grid, kBlock, 0, H[h].st>>>(a, b);
            e = hipGetLastError();
        }
    }
    if (two) {
        hipError_t j = hipEventRecord(ev_join, st2);
        if (j == hipSuccess) j = hipStreamWaitEvent(st, ev_join, 0);
        if (e == hipSuccess) e = j;
    }
    return e;
}

}  // namespace mcmc

// doubles of the row-layout u buffer per chain (64 NC)
int64_t mcmc_glm_ram_wave_ustride(int d) { return d <= 256 ? 256 : d <= 512 ? 512 : 1024; }

hipError_t mcmc_launch_glm_ram_wave(const mcmc::KernelArgs& a, double* u, double* nz, double* xprop, double* lpp,
                                    hipStream_t st, hipStream_t st2, hipEvent_t ev_fork, hipEvent_t ev_join) {
    using namespace mcmc;
    const GlmRamBufs b{u, nz, xprop, nullptr, mcmc_glm_ram_wave_ustride(a.s.d), 0};
    if (a.s.d <= 256) {                                       // two chains a wave (32 lanes each, 128 G rows)
        const int g = a.s.d <= 128 ? 1 : 2;
        mcmc_note_step_kernel("glm_ram_update<GlmHalfWaveChain<%d>, true>", g);
        return g == 1 ? glm_ram_wave_g<GlmHalfWaveChain<1>>(a, b, lpp, st, st2, ev_fork, ev_join)
                      : glm_ram_wave_g<GlmHalfWaveChain<2>>(a, b, lpp, st, st2, ev_fork, ev_join);
    }
    const int g = wpc_nb_for(a.s.d);
    mcmc_note_step_kernel("glm_ram_update<GlmWaveChain<%d>, true>", g);
    switch (g) {
        case 2: return glm_ram_wave_g<GlmWaveChain<2>>(a, b, lpp, st, st2, ev_fork, ev_join);
        case 4: return glm_ram_wave_g<GlmWaveChain<4>>(a, b, lpp, st, st2, ev_fork, ev_join);
        default: return hipErrorInvalidValue;
    }
}
