// ram_wave.hpp -- robust adaptive Metropolis (RAM.jl:41-79) for 32 < d <= 1024 on separable targets: the factor of
// each chain column-major in HBM, its rows spread over the lanes of the chain's wave (or half wave).  Included by
// kernels/wpc_ram.hip only.
//
// Storage.  One chain's factor is a block of ram_ld doubles (d(d+1)/2 rounded up to 8), column-major packed: column
// k holds rows k..d-1 from ram_wave_colstart(k) = k d - k(k-1)/2, so element (q, k) is at ram_wave_colstart(k) + q - k.
// Blocks are chain-major ([chain][ram_ld]), the second half of the ping-pong pair ram_hs doubles on.
//
// Row ownership (round 4).  Lane l of the chain's L lanes (L = 64: one chain a wave, WaveChain; L = 32: two chains a
// wave, HalfWaveChain) owns factor rows q = l + L s, s < NC: every buffer access of a column is L consecutive
// doubles per chain, one coalesced 256 / 512 B run.  (Rounds 2-3 gave lane l the rows of its own coordinates,
// 4 (l + L g) + e: each access then had a 32 B lane stride, and the texture addresser -- TA_BUSY_avr 1.00 of the
// dispatch in profiles/r04_pmc_ram256.md -- was what set the rate.)  The chain's vectors keep the coordinate
// ("quad") layout of the sampler policy: z and S z cross between the two layouts through LDS once per step
// (ram_to_rows / ram_to_quads), so the sums (|z|^2, the log-target) keep their order and the oracle its restatement.
// Column k's pivot u[k] and S[k][k] come from their owner lane k mod L by readlane; the next column's entries are
// loaded while this one is computed, with unconditional buffer accesses whose out-of-column lanes the range check
// masks (exact vmcnt waits, no wait on the previous column's stores).
#pragma once
#include "samplers.hpp"

namespace mcmc {

__host__ __device__ constexpr int64_t ram_wave_colstart(int64_t k, int64_t d) { return k * d - k * (k - 1) / 2; }

__device__ __forceinline__ double ram_readlane(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// the factor blocks of a wave's chains (one block, or the two adjacent blocks of a HalfWaveChain pair)
__device__ __forceinline__ ram_rsrc_t ram_chain_rsrc(const double* block, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(block), (short)0, (int)bytes, 0x00020000);
}

// column k's pivot entries from their owner lane j of each chain: one chain per wave (L = 64) reads lane j; two
// chains per wave (L = 32) read lanes j and 32 + j and each half takes its own
template <int L>
__device__ __forceinline__ double ram_bcast(double v, int j) {
    if constexpr (L == 64) {
        return ram_readlane(v, j);
    } else {
        const double a = ram_readlane(v, j), b = ram_readlane(v, j + 32);
        return (threadIdx.x & 32) ? b : a;
    }
}

// Unconditional buffer accesses whose lanes outside the column are masked by the buffer's range check: the whole
// byte offset rides in the vector offset, and a masked lane's is kRamOob, past any num_records (a chain pair's
// blocks are < 2 GB), so its load returns 0 and its store is dropped.  With no branch around them the compiler
// counts the memory operations exactly, and the wait for column k + 1's prefetched entries does not also wait
// for column k's stores (a masked, branched access makes it wait for everything: vmcnt(0)).
constexpr uint32_t kRamOob = 0xfffffff0u;
// columns of the factor in flight in ram_wave_update (1: the next column's loads issued before this one's update; 2:
// the next two)
#ifndef RAM_WAVE_PF
#define RAM_WAVE_PF 2
#endif
// 1 (default): a column's per-slot work starts at the owner's slot (the slots before hold rows above the pivot)
#ifndef RAM_WAVE_PRUNE
#define RAM_WAVE_PRUNE 1
#endif
__device__ __forceinline__ double ram_wload_m(ram_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ void ram_wstore_m(ram_rsrc_t r, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(ram_u32x2, v), r, off, 0, 0);
}

// The columns k = 0..d-1 in order: k = j + L s, owner lane j of the chain's L (runtime, wave-uniform), owner slot s
// (unrolled).  col(k, j, s) is called once per column.
template <int NC, int L, class F>
__device__ __forceinline__ void ram_wave_columns(int d, F&& col) {
#pragma unroll
    for (int s = 0; s < NC; ++s) {
        for (int j = 0; j < L; ++j) {
            const int k = j + L * s;
            if (k >= d) return;
            col(k, j, s);
        }
    }
}

// column k's entries of this lane's rows (q >= k, q < d; else 0); vo: the chain's block and the lane's row, bytes
template <int NC, int L>
__device__ __forceinline__ void ram_wave_load_col(ram_rsrc_t S, uint32_t vo, int lane, int d, int k, double (&v)[NC]) {
    const uint32_t base = vo + (uint32_t)(ram_wave_colstart(k, d) - k) * 8u;
#pragma unroll
    for (int s = 0; s < NC; ++s) {
        const int q = lane + L * s;
        v[s] = ram_wload_m(S, (q >= k && q < d) ? base + (uint32_t)(L * s) * 8u : kRamOob);   // 0 outside
    }
}

// u = S z in row layout (z in row layout): per row the fma chain over c = 0..q, one column at a time
template <int NC, int L>
__device__ __forceinline__ void ram_wave_matvec(ram_rsrc_t S, uint32_t vo, int lane, int d, const double (&z)[NC],
                                                double (&u)[NC]) {
#pragma unroll
    for (int s = 0; s < NC; ++s) u[s] = 0.0;
    ram_wave_columns<NC, L>(d, [&](int k, int j, int ks) {
        const double zk = ram_bcast<L>(z[ks], j);
        double v[NC];
        ram_wave_load_col<NC, L>(S, vo, lane, d, k, v);
#pragma unroll
        for (int s = 0; s < NC; ++s) {
            if (RAM_WAVE_PRUNE && s < ks) continue;            // rows L s .. L s + L - 1 < k: none takes column k
            const int q = lane + L * s;
            const double f = __builtin_fma(v[s], zk, u[s]);
            u[s] = (q >= k && q < d) ? f : u[s];
        }
    });
}

// ram_update for the wave layout (same operations per entry, same NEXT fold of the next step's S z, whose normals
// zn, row layout, are drawn beforehand); u, un in row layout
template <int NC, int L, bool NEXT>
__device__ __forceinline__ void ram_wave_update(ram_rsrc_t Ss, ram_rsrc_t Sd, uint32_t vo, int lane, int d,
                                                double alpha, double nz, double (&u)[NC],
                                                const double (&zn)[NC], double (&un)[NC]) {
    const double beta = alpha / nz;
    const bool up = beta >= 0.0;
    const double sb = __builtin_sqrt(__builtin_fabs(beta));
#pragma unroll
    for (int s = 0; s < NC; ++s) u[s] = sb * u[s];
    if (NEXT) {
#pragma unroll
        for (int s = 0; s < NC; ++s) un[s] = 0.0;
    }
    // column k's entries l0, the next RAM_WAVE_PF - 1 columns' loads in flight (the update is a chain over the
    // columns; the loads are not: more of them in flight is more of the factor's bandwidth)
    double l0[NC], l1[NC], lp2[NC];
    ram_wave_load_col<NC, L>(Ss, vo, lane, d, 0, l0);
    if (RAM_WAVE_PF > 1 && d > 1) ram_wave_load_col<NC, L>(Ss, vo, lane, d, 1, l1);
    ram_wave_columns<NC, L>(d, [&](int k, int j, int ks) {
        const uint32_t base = vo + (uint32_t)(ram_wave_colstart(k, d) - k) * 8u;
        if (RAM_WAVE_PF > 1) {
            if (k + 2 < d) ram_wave_load_col<NC, L>(Ss, vo, lane, d, k + 2, lp2);
        } else {
            if (k + 1 < d) ram_wave_load_col<NC, L>(Ss, vo, lane, d, k + 1, l1);
        }
        const double zk = NEXT ? ram_bcast<L>(zn[ks], j) : 0.0;
        const double lkk = ram_bcast<L>(l0[ks], j);
        const double xk = ram_bcast<L>(u[ks], j);
        const double t2 = xk * xk;
        const double l2 = lkk * lkk;
        const double r = __builtin_sqrt(up ? l2 + t2 : l2 - t2);
        const double cc = r / lkk;
        const double sn = xk / lkk;
        const double sns = up ? sn : -sn;
        const double ic = 1.0 / cc;
#pragma unroll
        for (int s = 0; s < NC; ++s) {
            // every slot from the owner's on computes (the slots before it hold rows above k: no entry of theirs
            // changes, so they are skipped, a compile-time bound of the unrolled owner slot); selects keep the
            // entries outside rows k..d-1 unchanged (the same values as per-row branches: row k takes r, rows below
            // take l)
            if (RAM_WAVE_PRUNE && s < ks) continue;
            const int q = lane + L * s;
            const bool diag = q == k, below = q > k && q < d;
            const double l = (l0[s] + sns * u[s]) * ic;
            const double out = diag ? r : l;
            ram_wstore_m(Sd, (diag || below) ? base + (uint32_t)(L * s) * 8u : kRamOob, out);
            const double un1 = __builtin_fma(out, zk, un[s]);
            if (NEXT) un[s] = (diag || below) ? un1 : un[s];
            const double u1 = cc * u[s] - sn * l;
            u[s] = below ? u1 : u[s];
        }
#pragma unroll
        for (int s = 0; s < NC; ++s) {
            if (RAM_WAVE_PRUNE && s < ks) continue;            // rows above every later column
            l0[s] = l1[s];
            if (RAM_WAVE_PF > 1) l1[s] = lp2[s];
        }
    });
}

// Coordinate (quad) layout <-> row layout of a chain's vector, through the wave's LDS slice: the policy's lane l
// slot 4 g + e holds coordinate 4 (l + L g) + e; the row layout's lane l slot s holds coordinate l + L s.  The slice
// is private to the wave (no barrier: LDS operations of one wave complete in order; the fences keep the compiler
// from moving them across each other).
template <int NC, int L>
__device__ __forceinline__ void ram_to_rows(double* slice, int lane, const double (&v)[NC], double (&r)[NC]) {
#pragma unroll
    for (int s = 0; s < NC; ++s) slice[4 * (lane + L * (s >> 2)) + (s & 3)] = v[s];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int s = 0; s < NC; ++s) r[s] = slice[lane + L * s];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
template <int NC, int L>
__device__ __forceinline__ void ram_to_quads(double* slice, int lane, const double (&r)[NC], double (&v)[NC]) {
#pragma unroll
    for (int s = 0; s < NC; ++s) slice[lane + L * s] = r[s];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int s = 0; s < NC; ++s) v[s] = slice[4 * (lane + L * (s >> 2)) + (s & 3)];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// Two chains per wave, 32 lanes per chain (RAM on separable targets, 32 < d <= 128 G; ram_wave_body): half h =
// lane >> 5 of wave w runs chain 2 w + h, lane l = lane & 31 of it owns coordinates 4 (l + 32 k) + e; sums per lane,
// then the butterfly over the half (oracle order ORC_ORDER_HALF).  The wave-uniform pivot work of a RAM column is
// then shared by two chains.
template <int G>
struct HalfWaveChain {
    static constexpr int NB = G;
    static constexpr int NC = 4 * G;
    static constexpr bool kPairs = false;
    static constexpr int L = 32;
    int64_t c;
    bool live;
    int d;
    int lane;
    int64_t ldr;
    BmTables<kTabGlobal, kBlock> bt;
    __device__ HalfWaveChain(const StepArgs& s) {
        c = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 2 + ((threadIdx.x >> 5) & 1);
        live = c < s.C;
        d = s.d;
        lane = (int)(threadIdx.x & 31);
        ldr = s.ld;
        bt.init();
    }
    __device__ __forceinline__ int coord(int k) const { return 4 * (lane + L * (k >> 2)) + (k & 3); }
    __device__ __forceinline__ bool valid(int k) const { return coord(k) < d; }
    __device__ __forceinline__ uint32_t block(int b) const { return (uint32_t)(lane + L * b); }
    __device__ __forceinline__ double reduce(double v) const {
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
        return v;
    }
    __device__ __forceinline__ bool any(bool v) const {
        const uint64_t m = __ballot(v);
        return ((threadIdx.x & 32) ? (m >> 32) : (m & 0xffffffffull)) != 0;
    }
    __device__ __forceinline__ void load(const double* x, int64_t /*ld*/, double (&v)[NC]) const {
        const double* row = x + (size_t)(live ? c : 0) * (size_t)ldr;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int j0 = 4 * (lane + L * g);
            if (j0 < d) {
                const double4 q = *reinterpret_cast<const double4*>(row + j0);
                v[4 * g] = q.x; v[4 * g + 1] = q.y; v[4 * g + 2] = q.z; v[4 * g + 3] = q.w;
            } else {
                v[4 * g] = v[4 * g + 1] = v[4 * g + 2] = v[4 * g + 3] = 0.0;
            }
        }
#pragma unroll
        for (int k = 0; k < NC; ++k)
            if (!valid(k)) v[k] = 0.0;
    }
    __device__ __forceinline__ void store(double* x, int64_t /*ld*/, const double (&v)[NC]) const {
        if (!live) return;
        double* row = x + (size_t)c * (size_t)ldr;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int j0 = 4 * (lane + L * g);
            if (j0 < d) *reinterpret_cast<double4*>(row + j0) = make_double4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
        }
    }
    __device__ __forceinline__ double load_scalar(const double* p) const { return p[live ? c : 0]; }
    template <class T>
    __device__ __forceinline__ void store_t(T* p, T v) const {
        if (live && lane == 0) p[c] = v;
    }
    // kept sample into the chain-major staging layout [nkept][C][ldr], as WaveChain
    __device__ __forceinline__ void store_kept(const StepArgs& s, int64_t kk, const double (&v)[NC],
                                               double* base) const {
        if (base == nullptr || !live) return;
        double* row = base + ((size_t)kk * (size_t)s.C + (size_t)c) * (size_t)ldr;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int j0 = 4 * (lane + L * g);
            if (j0 < d) *reinterpret_cast<double4*>(row + j0) = make_double4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
        }
    }
    __device__ __forceinline__ void count_evals(const StepArgs& s, int64_t n) const {
        if (s.n_evals != nullptr && live && lane == 0) atomicAdd(s.n_evals, (unsigned long long)n);
    }
    // the wave's two chains (2 w, 2 w + 1) are adjacent bits of one accept word: one atomicOr per wave
    __device__ __forceinline__ void store_bit(const StepArgs& s, int64_t kk, bool acc) const {
        const uint64_t m = __ballot(acc && live && lane == 0);
        const uint64_t bits = (m & 1ull) | ((m >> 31) & 2ull);
        if ((threadIdx.x & 63) == 0 && bits != 0 && s.acc_bits != nullptr)
            atomicOr((unsigned long long*)&s.acc_bits[(size_t)kk * (size_t)s.nw + (size_t)(c >> 6)], bits << (c & 63));
    }
};

// Robust adaptive Metropolis for 32 < d <= 1024, wave per chain (the layout above): the lane-per-chain body's steps
// with the factor's rows spread over the chain's lanes.
template <class P, class M>
__device__ __forceinline__ void ram_wave_body(const KernelArgs& a) {
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const P p(s);
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    constexpr int NC = P::NC;
    constexpr int L = P::L;               // lanes per chain: 64 (WaveChain) or 32 (HalfWaveChain, two chains a wave)
    constexpr int CPW = 64 / L;
    const int d = s.d;
    const int64_t cu = (int64_t)blockIdx.x * (kBlock / 64) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (cu * CPW >= s.C) return;          // a tail wave with no live chain (no barriers below: it may leave)
    // the wave's LDS slice for the layout changes (L NC doubles per chain), and where x waits out the factor update
    // (the update holds the column's entries, u, the next S z and its normals: x would take the registers that
    // let three waves share a SIMD)
    __shared__ double xpose[kBlock / 64][64 * NC];
    __shared__ double xpark[kBlock / 64][NC][64];
    double* const slice = &xpose[threadIdx.x >> 6][((threadIdx.x & 63) / L) * L * NC];
    double (*const park)[64] = xpark[threadIdx.x >> 6];
    double x[NC];
    p.load(a.st.x, s.ld, x);
    double lp = p.load_scalar(a.st.lp);
    // the factor blocks of the wave's chains in each half: chains CPW w .. CPW w + CPW - 1 are adjacent blocks (the
    // runtime allocates round_up(C, 8) of them), one buffer resource over them, the chain's block and the lane's
    // row by the vector offset
    const int64_t ld = a.st.ram_ld;
    double* const B0 = a.st.ram_L + (uint64_t)(cu * CPW) * (uint64_t)ld;
    const uint64_t hs = (uint64_t)a.st.ram_hs;
    const int64_t rbytes = ld * 8 * CPW;
    const int lane = p.lane;
    const uint32_t vo = (uint32_t)((threadIdx.x & 63) / L) * (uint32_t)(ld * 8) + (uint32_t)lane * 8;
    double u[NC], uq[NC], nz;             // S z: row layout (u) and coordinate layout (uq)
    if (s.nsteps > 0) {
        const int64_t i = s.step_begin;
        double z[NC], zr[NC];
        gen_normals(p, rs, chain, (uint32_t)i, z);
        double a2 = 0.0;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (!p.valid(k)) z[k] = 0.0;
            a2 = __builtin_fma(z[k], z[k], a2);                               // dot(rvec, rvec)
        }
        nz = p.reduce(a2);
        ram_to_rows<NC, L>(slice, lane, z, zr);
        ram_wave_matvec<NC, L>(ram_chain_rsrc(B0 + (uint64_t)((i - 1) & 1) * hs, rbytes), vo, lane, d, zr, u);
        ram_to_quads<NC, L>(slice, lane, u, uq);
    }
    Keeper keep(s);
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        double lpp;
        {
            double xp[NC];
#pragma unroll
            for (int k = 0; k < NC; ++k) xp[k] = x[k] + uq[k];                // RAM.jl:60
            bool oos;
            lpp = eval_lp(p, model, xp, oos);
        }
        const double ratio = lpp - lp;
        const bool acc = mh_accept_short_circuit(rs, chain, (uint32_t)i, ratio);
        if (acc) {
#pragma unroll
            for (int k = 0; k < NC; ++k) x[k] = x[k] + uq[k];
            lp = lpp;
        }
        int64_t kk;
        if (keep.take(i, &kk)) {
            p.store_kept(s, kk, x, s.samples);
            p.store_bit(s, kk, acc);
        }
        const double alpha = ram_alpha(i, d, ratio, sa.rate);
        const ram_rsrc_t Ss = ram_chain_rsrc(B0 + (uint64_t)((i - 1) & 1) * hs, rbytes);
        const ram_rsrc_t Sd = ram_chain_rsrc(B0 + (uint64_t)(i & 1) * hs, rbytes);
        if (t + 1 < s.nsteps) {
            double zn[NC], znr[NC], un[NC];
            gen_normals(p, rs, chain, (uint32_t)(i + 1), zn);                  // step i + 1's rvec
            double a2 = 0.0;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                if (!p.valid(k)) zn[k] = 0.0;
                a2 = __builtin_fma(zn[k], zn[k], a2);
            }
            ram_to_rows<NC, L>(slice, lane, zn, znr);
#pragma unroll
            for (int k = 0; k < NC; ++k) park[k][threadIdx.x & 63] = x[k];
            ram_wave_update<NC, L, true>(Ss, Sd, vo, lane, d, alpha, nz, u, znr, un);
#pragma unroll
            for (int k = 0; k < NC; ++k) x[k] = park[k][threadIdx.x & 63];
#pragma unroll
            for (int k = 0; k < NC; ++k) u[k] = un[k];
            ram_to_quads<NC, L>(slice, lane, u, uq);
            nz = p.reduce(a2);
        } else {
            double zn[NC], un[NC];
            ram_wave_update<NC, L, false>(Ss, Sd, vo, lane, d, alpha, nz, u, zn, un);
        }
    }
    p.store(a.st.x, s.ld, x);
    p.store_t(a.st.lp, lp);
    p.count_evals(s, s.nsteps);
}

}  // namespace mcmc
