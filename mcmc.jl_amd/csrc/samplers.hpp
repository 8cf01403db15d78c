// samplers.hpp -- fused multi-step sampler kernels, generic over the chain->lane mapping.
//
// A kernel launch advances every chain by `nsteps` steps of the SerialMC loop
// (SerialMC.jl:47-67) with the chain state held in VGPRs; HBM sees the state
// once per launch plus the kept samples/gradients and the accept bits.
//
// Two mappings (policies) share the step code:
//   LaneChain<NB>  one thread = one chain, coordinates j = 0..4NB-1 in registers,
//                  state SoA x[j][c] (coalesced across the wave), sums in order
//                  j = 0,1,... (oracle order 0).  d <= 32.
//   WaveChain<G>   one wave = one chain, lane l owns coordinates 4(l+64k)+e
//                  (k < G, e < 4), state chain-major x[c][j] read as 2 x 16 B per
//                  lane, sums = per-lane partial then xor butterfly over the wave
//                  (oracle order 1).  32 < d <= 2048.
// Both draw coordinate j's normal from Philox block j/4, slot j%4 of
// (chain, step, block, TAG_NORMAL), so the chain's random stream does not
// depend on the mapping.
//
// Per step (reference file:line for each sampler):
//   RWM    RWM.jl:58-71      x' = x + randn .* scale; accept iff r > 0 || r > log(rand())
//   MALA   MALA.jl:89-125    Langevin proposal, forward/backward densities, EmpMCTuner
//   HMC    HMC.jl:126-173    L leapfrogs (HMC.jl:93-102), accept iff rand() < exp(H0 - H)
//   HMCDA  HMCDA.jl:97-142   nLeaps = max(1, round(len/eps)), p = min(1, exp(H0-H)),
//                            dual averaging while i < burnin
#pragma once
#include "common.hpp"
#include "detmath.hpp"
#include "models.hpp"
#include "ram.hpp"
#include "host/kernels_api.hpp"

namespace mcmc {

constexpr int kBlock = 256;

// Where a kernel reads the Box-Muller tables (the radius polynomials of bm_radius_u32 and the angle table):
//   kTabLds     staged once per block into LDS (56 KB: the hot kernels -- their per-lane row gathers go to LDS);
//   kTabGlobal  straight from global memory (L1 / L2), for kernels whose occupancy 56 KB per block would cut or
//               whose LDS is taken (the few-chain kernels, RAM, the diagnostics); the same values either way.
enum TabMode : int { kTabLds = 0, kTabGlobal = 1 };

struct BmLds {
    double (*rd)[2];
    double (*sc)[2];
};
// The block's LDS copies (one allocation per kernel, whoever asks)
__device__ __forceinline__ BmLds bm_lds_tables() {
    __shared__ __attribute__((aligned(16))) double lds_radd[4 * BM_RADP_NROWS][2];
    __shared__ __attribute__((aligned(16))) double lds_sct[1024][2];
    return BmLds{lds_radd, lds_sct};
}

// The tables into a block's LDS by its NT threads: every 16-byte load of a batch in flight before its first store
// (a loop of load-store pairs costs one L2 round trip per iteration), then one barrier.
template <int NT>
__device__ __forceinline__ void stage_bm_tables(const BmLds& L) {
    typedef double f64x2_t __attribute__((ext_vector_type(2)));
    constexpr int kD = 4 * BM_RADP_NROWS, kS = 1024;     // 16-byte units of each table
    constexpr int kU = kD + kS;
    constexpr int kN = (kU + NT - 1) / NT;
    constexpr int kBatch = 8;
    const f64x2_t* gd = reinterpret_cast<const f64x2_t*>(&kBmRadPTab[0][0]);
    const f64x2_t* gs = reinterpret_cast<const f64x2_t*>(&kBmSinCos1024Tab[0][0]);
    f64x2_t* ld = reinterpret_cast<f64x2_t*>(&L.rd[0][0]);
    f64x2_t* ls = reinterpret_cast<f64x2_t*>(&L.sc[0][0]);
#pragma unroll
    for (int j0 = 0; j0 < kN; j0 += kBatch) {
        f64x2_t v[kBatch];
#pragma unroll
        for (int j = j0; j < j0 + kBatch && j < kN; ++j) {
            const int u = (int)threadIdx.x + NT * j;
            if (u < kU) v[j - j0] = u < kD ? gd[u] : gs[u - kD];
        }
#pragma unroll
        for (int j = j0; j < j0 + kBatch && j < kN; ++j) {
            const int u = (int)threadIdx.x + NT * j;
            if (u < kD) ld[u] = v[j - j0];
            else if (u < kU) ls[u - kD] = v[j - j0];
        }
    }
    __syncthreads();
}

// The tables a policy reads: LDS (staged by stage()) or global
template <int TAB, int NT>
struct BmTables {
    RadTab rad;
    const double (*sct)[2];
    BmLds lds;
    __device__ __forceinline__ void init() {
        if constexpr (TAB == kTabLds) {
            lds = bm_lds_tables();
            rad = RadTab{lds.rd, true};
            sct = lds.sc;
        } else {
            rad = rad_tab_global();
            sct = kBmSinCos1024Tab;
        }
    }
    __device__ __forceinline__ void stage() const {
        if constexpr (TAB == kTabLds) stage_bm_tables<NT>(lds);
    }
};

// ------------------------------------------------------------------ mappings
// NB = ceil(d/4).  FULL: d == 4 NB, every register coordinate is a real one -- no validity masks
// (with a runtime d they are per-coordinate uniform masks, which overflow the SGPR file at NB = 8).
// SPLIT: eval_lp sums in PairChain's order (coordinates of the first PairChain half, then the second, then the two
// partial sums added) -- for the few-chain RWM kernel lpc_rwm_la, which runs the same chains as the 16 < d <= 32
// PairChain kernels and must agree with them bit for bit
// TH: threads per block (chains per block); TAB: where the Box-Muller tables are read (TabMode)
template <int NB_, bool FULL = false, bool SPLIT = false, int TH = kBlock, int TAB = kTabGlobal>
struct LaneChain {
    static constexpr int NB = NB_;
    static constexpr int NC = 4 * NB_;
    static constexpr int kSplit = SPLIT ? 4 * ((NB_ + 1) / 2) : 0;
    static constexpr int kThreads = TH;
    static constexpr int kChainsPerBlock = TH;
    static constexpr bool kPairs = false;
    int64_t c;        // local chain index
    bool live;        // c < C
    int d;
    BmTables<TAB, TH> bt;     // the Box-Muller tables (every block thread calls the constructor)
    // defer: the caller issues its state loads first and then calls stage() (the two latencies overlap)
    __device__ LaneChain(const StepArgs& s, bool defer = false) {
        c = (int64_t)blockIdx.x * TH + threadIdx.x;
        live = c < s.C;
        d = s.d;
        bt.init();
        if (!defer) stage();
    }
    __device__ __forceinline__ void stage() const { bt.stage(); }
    __device__ __forceinline__ int coord(int k) const { return k; }
    // blocks 0..NB-2 are always full (NB = ceil(d/4)); only the last block's coordinates are tested
    __device__ __forceinline__ bool valid(int k) const { return FULL || k < 4 * (NB - 1) || k < d; }
    __device__ __forceinline__ uint32_t block(int b) const { return (uint32_t)b; }
    __device__ __forceinline__ double reduce(double v) const { return v; }
    __device__ __forceinline__ bool any(bool v) const { return v; }
    // running addresses (see store_kept): no per-coordinate uniform offsets live across the step loop
    // (the opaque value is the element offset, not the pointer, so the accesses stay global_*, not flat_*)
    __device__ __forceinline__ void load(const double* x, int64_t ld, double (&v)[NC]) const {
        uint64_t o = (uint64_t)(live ? c : 0);
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            v[k] = valid(k) ? x[o] : 0.0;
            o += (uint64_t)ld;
            asm volatile("" : "+v"(o));
        }
    }
    __device__ __forceinline__ void store(double* x, int64_t ld, const double (&v)[NC]) const {
        if (!live) return;
        uint64_t o = (uint64_t)c;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (valid(k)) x[o] = v[k];
            o += (uint64_t)ld;
            asm volatile("" : "+v"(o));
        }
    }
    __device__ __forceinline__ double load_scalar(const double* p) const { return p[live ? c : 0]; }
    template <class T>
    __device__ __forceinline__ T load_t(const T* p) const { return p[live ? c : 0]; }
    template <class T>
    __device__ __forceinline__ void store_t(T* p, T v) const {
        if (live) p[c] = v;
    }
    // kept sample in the C ABI layout [nkept][d][C]
    __device__ __forceinline__ void store_kept(const StepArgs& s, int64_t kk, const double (&v)[NC],
                                               double* base) const {
        if (base == nullptr || !live) return;
        double* p = base + (size_t)kk * (size_t)d * (size_t)s.C;
        const uint64_t C = (uint64_t)s.C;
        uint64_t o = (uint64_t)c;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (valid(k)) p[o] = v[k];
            o += C;
            // one running offset: otherwise the NC uniform offsets k*C are precomputed and held in
            // SGPRs across the step loop, spilling the scalar file
            asm volatile("" : "+v"(o));
        }
    }
    // storeLeaps records, coordinate-major [l][d][C]: the kept-sample layout
    __device__ __forceinline__ void store_cm(const StepArgs& s, int64_t l, const double (&v)[NC], double* base) const {
        store_kept(s, l, v, base);
    }
    // add this chain's evaluation count to the launch-wide counter (one atomic per wave)
    __device__ __forceinline__ void count_evals(const StepArgs& s, int64_t n) const {
        if (s.n_evals == nullptr) return;
        unsigned long long v = live ? (unsigned long long)n : 0ull;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(s.n_evals, v);
    }
    __device__ __forceinline__ void store_bit(const StepArgs& s, int64_t kk, bool acc) const {
        const uint64_t mask = __ballot(acc && live);
        if ((threadIdx.x & 63) == 0 && s.acc_bits != nullptr) {
            const int64_t w = c >> 6;
            if (w < s.nw) s.acc_bits[(size_t)kk * (size_t)s.nw + (size_t)w] = mask;
        }
    }
};

// Two lanes per chain (16 < d <= 32): lane l of a wave holds half h = l >> 5 of chain (l & 31) of the wave's 32
// chains -- coordinates h NC .. h NC + NC - 1 (NC = 4 NB, NB = ceil(ceil(d/4) / 2) Philox blocks per lane) -- so a
// lane carries half the state and proposal of LaneChain and the kernel fits four waves per SIMD instead of two
// (the VALU issue rate of a SIMD grows with the waves it can pick from; scripts/probe_valu_rates.hip).  Sums: each
// lane accumulates its coordinates left to right, then (half 0) + (half 1), formed identically in both lanes by
// one v_permlane32_swap per dword (oracle order ORC_ORDER_PAIR).  Both lanes of a chain hold the same lp, ratio
// and accept decision; memory: row k of the wave's 32 chains is one 256-byte run per half.
template <int NB_, bool FULL = false, int TH = 512, int TAB = kTabLds>
struct PairChain {
    static constexpr int NB = NB_;
    static constexpr int NC = 4 * NB_;
    static constexpr int kThreads = TH;
    static constexpr int kChainsPerBlock = TH / 2;
    static constexpr bool kPairs = true;
    int64_t c;        // local chain index
    bool live;
    int d;
    int h;            // half: 0 (lanes 0-31) or 1 (lanes 32-63)
    BmTables<TAB, TH> bt;
    __device__ PairChain(const StepArgs& s, bool defer = false) {
        const int lane = (int)(threadIdx.x & 63);
        c = (int64_t)blockIdx.x * kChainsPerBlock + (int64_t)(threadIdx.x >> 6) * 32 + (lane & 31);
        h = lane >> 5;
        live = c < s.C;
        d = s.d;
        bt.init();
        if (!defer) stage();
    }
    __device__ __forceinline__ void stage() const { bt.stage(); }
    // the chain index as of this point: addresses formed from it after the step loop (state, lp) or on a kept step
    // (accept bits) cannot be hoisted ahead of the loop and held -- at the 128-VGPR budget the held 64-bit addresses
    // were spilled to scratch (3 x 8 B per lane, ~100 MB of scratch traffic per 2^20-chain launch)
    __device__ __forceinline__ static uint32_t tid_now() {
        uint32_t t = threadIdx.x;
        asm volatile("" : "+v"(t));
        return t;
    }
    __device__ __forceinline__ int64_t c_now() const {
        const uint32_t t = tid_now();
        return (int64_t)blockIdx.x * kChainsPerBlock + (int64_t)((t >> 6) * 32 + (t & 31));
    }
    __device__ __forceinline__ int coord(int k) const { return h * NC + k; }
    __device__ __forceinline__ bool valid(int k) const { return FULL || coord(k) < d; }
    __device__ __forceinline__ uint32_t block(int b) const { return (uint32_t)(h * NB + b); }
    // half `which`'s value of v in both lanes of the chain (v_permlane32_swap: {half 0's, half 1's} broadcasts)
    __device__ __forceinline__ double from_half(double v, int which) const {
        const uint64_t u = (uint64_t)__double_as_longlong(v);
        const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
        const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        return which == 0 ? __longlong_as_double((long long)(((uint64_t)b[0] << 32) | a[0]))
                          : __longlong_as_double((long long)(((uint64_t)b[1] << 32) | a[1]));
    }
    // (half 0's value) + (half 1's value) in both lanes of the chain, bitwise the same
    __device__ __forceinline__ double reduce(double v) const {
        const uint64_t u = (uint64_t)__double_as_longlong(v);
        const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
        const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);   // {half 0's, half 1's}
        const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        const double v0 = __longlong_as_double((long long)(((uint64_t)b[0] << 32) | a[0]));
        const double v1 = __longlong_as_double((long long)(((uint64_t)b[1] << 32) | a[1]));
        return v0 + v1;
    }
    __device__ __forceinline__ bool any(bool v) const {
        const uint64_t m = __ballot(v);
        const int l = (int)(threadIdx.x & 31);
        return (((m >> l) | (m >> (l + 32))) & 1ull) != 0;
    }
    __device__ __forceinline__ void load(const double* x, int64_t ld, double (&v)[NC]) const {
        uint64_t o = (uint64_t)(live ? c : 0) + (uint64_t)(h * NC) * (uint64_t)ld;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            v[k] = valid(k) ? x[o] : 0.0;
            o += (uint64_t)ld;
            asm volatile("" : "+v"(o));
        }
    }
    __device__ __forceinline__ void store(double* x, int64_t ld, const double (&v)[NC]) const {
        if (!live) return;
        const int hn = (int)((tid_now() >> 5) & 1);
        uint64_t o = (uint64_t)c_now() + (uint64_t)(hn * NC) * (uint64_t)ld;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (valid(k)) x[o] = v[k];
            o += (uint64_t)ld;
            asm volatile("" : "+v"(o));
        }
    }
    __device__ __forceinline__ double load_scalar(const double* p) const { return p[live ? c : 0]; }
    template <class T>
    __device__ __forceinline__ T load_t(const T* p) const { return p[live ? c : 0]; }
    template <class T>
    __device__ __forceinline__ void store_t(T* p, T v) const {
        if (live && h == 0) p[c_now()] = v;
    }
    __device__ __forceinline__ void store_kept(const StepArgs& s, int64_t kk, const double (&v)[NC],
                                               double* base) const {
        if (base == nullptr || !live) return;
        // row (h NC + k) of sample kk: a wave-uniform row base (scalar registers) plus the lane's 32-bit byte offset
        // (chain and half; a sample is d C doubles, far below 4 GiB), so each store is a saddr global_store with
        // no per-lane 64-bit address arithmetic
        const uint64_t C = (uint64_t)s.C;
        const uint32_t lo = (uint32_t)((uint64_t)c * 8u + (uint64_t)(h * NC) * C * 8u);
        char* row = reinterpret_cast<char*>(base + (size_t)kk * (size_t)d * (size_t)C);
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (valid(k)) *reinterpret_cast<double*>(row + lo) = v[k];
            row += C * 8u;
        }
    }
    __device__ __forceinline__ void store_cm(const StepArgs& s, int64_t l, const double (&v)[NC], double* base) const {
        store_kept(s, l, v, base);
    }
    __device__ __forceinline__ void count_evals(const StepArgs& s, int64_t n) const {
        if (s.n_evals == nullptr) return;
        unsigned long long v = (live && h == 0) ? (unsigned long long)n : 0ull;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(s.n_evals, v);
    }
    // the wave's 32 chains are one half-word of an accept-bit word (bit c % 64 of word c / 64, little-endian)
    __device__ __forceinline__ void store_bit(const StepArgs& s, int64_t kk, bool acc) const {
        const uint64_t mask = __ballot(acc && live);
        if ((threadIdx.x & 63) == 0 && s.acc_bits != nullptr) {
            const int64_t cc = c_now();
            const int64_t w = cc >> 6;
            if (w < s.nw)
                reinterpret_cast<uint32_t*>(s.acc_bits)[((size_t)kk * (size_t)s.nw + (size_t)w) * 2 + (size_t)((cc >> 5) & 1)] =
                    (uint32_t)mask;
        }
    }
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

// Sum of a per-chain quantity over the W waves of a block-per-chain kernel: each wave's butterfly, then the wave
// sums left to right (oracle order W); two barriers (the partials buffer is reused by the next call)
template <int W>
__device__ __forceinline__ double block_sum(double v) {
    v = wave_sum(v);
    if (W == 1) return v;
    __shared__ double part[W];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = part[0];
#pragma unroll
    for (int w = 1; w < W; ++w) t = t + part[w];
    __syncthreads();
    return t;
}

// FULL: d == 256 G W, every lane coordinate is a real one -- no per-coordinate validity masks (with a
// runtime d they are 4 G lane masks live across the step loop, which spill the scalar file)
// W > 1: one chain per block of W waves (d up to 256 G W; kernels/wpc_impl.hpp bpc_*): lane l of the 64 W owns
// coordinates 4 (l + 64 W k) + e, sums per lane, per wave, then over the waves (block_sum, oracle order W)
template <int G, bool FULL = false, int W = 1, int TAB = kTabGlobal>
struct WaveChain {
    static constexpr int NB = G;
    static constexpr int NC = 4 * G;
    static constexpr bool kPairs = false;
    static constexpr int L = 64 * W;                    // lanes per chain
    int64_t c;
    bool live;
    int d;
    int lane;
    int64_t ldr;      // row stride of chain-major state (multiple of 4)
    BmTables<TAB, W == 1 ? kBlock : 64 * W> bt;
    __device__ WaveChain(const StepArgs& s, bool defer = false) {
        c = W == 1 ? (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6) : (int64_t)blockIdx.x;
        live = c < s.C;
        d = s.d;
        lane = W == 1 ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
        ldr = s.ld;
        bt.init();
        if (!defer) stage();
    }
    __device__ __forceinline__ void stage() const { bt.stage(); }
    __device__ __forceinline__ int coord(int k) const { return 4 * (lane + L * (k >> 2)) + (k & 3); }
    __device__ __forceinline__ bool valid(int k) const { return FULL || coord(k) < d; }
    __device__ __forceinline__ uint32_t block(int b) const { return (uint32_t)(lane + L * b); }
    __device__ __forceinline__ double reduce(double v) const { return block_sum<W>(v); }
    __device__ __forceinline__ bool any(bool v) const { return W == 1 ? __ballot(v) != 0 : __syncthreads_or(v) != 0; }
    __device__ __forceinline__ void load(const double* x, int64_t /*ld*/, double (&v)[NC]) const {
        const double* row = x + (size_t)(live ? c : 0) * (size_t)ldr;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int j0 = 4 * (lane + L * g);
            if (FULL || j0 < d) {
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
            if (FULL || j0 < d) *reinterpret_cast<double4*>(row + j0) = make_double4(v[4 * g], v[4 * g + 1], v[4 * g + 2],
                                                                               v[4 * g + 3]);
        }
    }
    __device__ __forceinline__ double load_scalar(const double* p) const { return p[live ? c : 0]; }
    template <class T>
    __device__ __forceinline__ T load_t(const T* p) const { return p[live ? c : 0]; }
    template <class T>
    __device__ __forceinline__ void store_t(T* p, T v) const {
        if (live && lane == 0) p[c] = v;
    }
    // kept sample into the chain-major staging layout [nkept][C][ldr] (transposed to the C ABI
    // layout after the step loop)
    __device__ __forceinline__ void store_kept(const StepArgs& s, int64_t kk, const double (&v)[NC],
                                               double* base) const {
        if (base == nullptr || !live) return;
        double* row = base + ((size_t)kk * (size_t)s.C + (size_t)c) * (size_t)ldr;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int j0 = 4 * (lane + L * g);
            if (FULL || j0 < d) *reinterpret_cast<double4*>(row + j0) = make_double4(v[4 * g], v[4 * g + 1], v[4 * g + 2],
                                                                               v[4 * g + 3]);
        }
    }
    __device__ __forceinline__ void count_evals(const StepArgs& s, int64_t n) const {
        if (s.n_evals != nullptr && live && lane == 0) atomicAdd(s.n_evals, (unsigned long long)n);
    }
    // storeLeaps records, coordinate-major [l][d][C] (scattered 8-byte stores: a diagnostic, not a hot path)
    __device__ __forceinline__ void store_cm(const StepArgs& s, int64_t l, const double (&v)[NC], double* base) const {
        if (base == nullptr || !live) return;
        double* p = base + (size_t)l * (size_t)d * (size_t)s.C + (size_t)c;
#pragma unroll
        for (int k = 0; k < NC; ++k)
            if (valid(k)) p[(size_t)coord(k) * (size_t)s.C] = v[k];
    }
    __device__ __forceinline__ void store_bit(const StepArgs& s, int64_t kk, bool acc) const {
        if (live && lane == 0 && acc && s.acc_bits != nullptr)
            atomicOr((unsigned long long*)&s.acc_bits[(size_t)kk * (size_t)s.nw + (size_t)(c >> 6)],
                     1ull << (c & 63));
    }
};

// ------------------------------------------------------------------ shared pieces
template <class P>
__device__ __forceinline__ void gen_normals(const P& p, const Stream& rs, uint32_t chain, uint32_t step,
                                            double (&z)[P::NC]) {
#pragma unroll
    for (int b = 0; b < P::NB; ++b) {
        const u32x4 w = rs.block_us(chain, step, p.block(b), TAG_NORMAL);
        normals4(w, z[4 * b], z[4 * b + 1], z[4 * b + 2], z[4 * b + 3], p.bt.rad, p.bt.sct);
    }
}


template <class P>
struct split_of { static constexpr int value = 0; };
template <int NB, bool F, bool S, int T, int TAB>
struct split_of<LaneChain<NB, F, S, T, TAB>> { static constexpr int value = LaneChain<NB, F, S, T, TAB>::kSplit; };

template <class P, class M>
__device__ __forceinline__ double eval_lp(const P& p, const M& model, const double (&v)[P::NC], bool& oos) {
    if constexpr (is_joint<M>::value) return model.joint_lp(v, oos);    // a joint target (lane per chain)
    constexpr int S = split_of<P>::value;
    if constexpr (S > 0) {                              // LaneChain SPLIT: PairChain's order (see LaneChain)
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int k = 0; k < P::NC; ++k)
            if (p.valid(k)) {
                if (k < S) model.acc(a, v[k]);
                else model.acc(b, v[k]);
            }
        return llacc_finish(model, a + b, oos);
    }
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < P::NC; ++k)
        if (p.valid(k)) model.acc(a, v[k]);
    return llacc_finish(model, p.reduce(a), oos);
}

// The model's gradient at a point v, coordinate by coordinate: for a separable model the rule of coordinate k at
// the use (g(k, v[k]) is model.grad(v[k]), the code as before); for a joint model (is_joint) the whole gradient,
// formed once when need is set (a point out of support never reads it)
template <class M, int NC, bool J = is_joint<M>::value>
struct GradAt {
    const M& m;
    __device__ __forceinline__ GradAt(const M& model, const double (&)[NC], bool = true) : m(model) {}
    __device__ __forceinline__ double operator()(int, double v) const { return m.grad(v); }
};
template <class M, int NC>
struct GradAt<M, NC, true> {
    double g[NC];
    __device__ __forceinline__ GradAt(const M& model, const double (&v)[NC], bool need = true) {
        if (need) {
            model.joint_grad(v, g);
        } else {
#pragma unroll
            for (int k = 0; k < NC; ++k) g[k] = 0.0;
        }
    }
    __device__ __forceinline__ double operator()(int k, double) const { return g[k]; }
};

template <class P>
__device__ __forceinline__ double half_dot(const P& p, const double (&m)[P::NC]) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < P::NC; ++k)
        if (p.valid(k)) a = __builtin_fma(m[k], m[k], a);
    return 0.5 * p.reduce(a);
}

__device__ __forceinline__ bool mh_accept_short_circuit(const Stream& rs, uint32_t chain, uint32_t step, double ratio) {
    // RWM.jl:63 / MALA.jl:108: ratio > 0 || ratio > log(rand()); the uniform is drawn only if needed.
    bool acc = ratio > 0.0;
    if (!acc) {
        const u32x4 w = rs.block(chain, step, 0u, TAG_ACCEPT);
        acc = gt_det_log(ratio, uniform52(w.x, w.y));
    }
    return acc;
}

// The RWM / MALA test of step i (launch step t), RWM.jl:63 / MALA.jl:108.  PairChain: both lanes of a chain need
// the same uniform, so on even t the two halves draw steps i (half 0) and i + 1 (half 1) from the counter-based
// stream at once; half 0's draw is broadcast now and half 1's kept for step t + 1 -- one Philox block per chain per
// two steps, the same values as mh_accept_short_circuit's conditional draw (the stream is keyed by (chain, step)).
template <class P>
struct AcceptDraw {
    double u_next = 0.0;
    __device__ __forceinline__ bool test(const P& p, const Stream& rs, uint32_t chain, int64_t i, int t, double ratio) {
        if constexpr (P::kPairs) {
            double u;
            if ((t & 1) == 0) {
                const u32x4 w = rs.block(chain, (uint32_t)(i + p.h), 0u, TAG_ACCEPT);
                const double uu = uniform52(w.x, w.y);
                u = p.from_half(uu, 0);
                u_next = uu;
            } else {
                u = p.from_half(u_next, 1);
            }
            bool acc = ratio > 0.0;
            if (!acc) acc = gt_det_log(ratio, u);
            return acc;
        } else {
            return mh_accept_short_circuit(rs, chain, (uint32_t)i, ratio);
        }
    }
};

// tuner adaptation factor (MALA.jl:36-39, HMC.jl:165-169)
__device__ __forceinline__ double tune_factor(int32_t acc, int32_t prop, double target) {
    const double rate = (double)acc / (double)prop;
    return 1.0 / (1.0 + det_exp(-11.0 * (rate - target))) + 0.5;
}

// The kept steps of a launch (kept_index's set: local index burnin + 1 + m thinning, <= len) as a scalar
// cursor: one 64-bit scalar compare a step instead of kept_index's 64-bit remainder and signed compares, which
// the step loop ran on the VALU (a uniform 64-bit division and i64 compares have no scalar instructions).
struct Keeper {
    int64_t next;       // the next kept step (absolute index); -1: none left in this launch
    int64_t kk;         // its kept index
    int64_t thin;
    int32_t left;       // kept steps after next
    __device__ explicit Keeper(const StepArgs& s) {
        thin = s.thinning;
        const int64_t lo = s.step_begin - s.run_step0;                 // local index of the launch's first step
        const int64_t hi = lo + s.nsteps - 1;
        int64_t first = s.burnin + 1;
        if (lo > first) first += ((lo - first + thin - 1) / thin) * thin;
        const int64_t last = hi < s.len ? hi : s.len;
        if (first > last) {
            next = -1; kk = 0; left = 0;
        } else {
            next = s.run_step0 + first;
            kk = (first - s.burnin - 1) / thin;
            left = (int32_t)((last - first) / thin);
        }
    }
    // kept_index(i - run_step0, ...) for the launch's steps in order
    __device__ __forceinline__ bool take(int64_t i, int64_t* out) {
        if (i != next) return false;
        *out = kk;
        if (left > 0) { next += thin; kk += 1; left -= 1; } else next = -1;
        return true;
    }
};

// ------------------------------------------------------------------ RWM
// US: every coordinate has the same scale (s.scale1), held in one SGPR pair instead of d of them
template <class P, class M, bool US = false>
__device__ __forceinline__ void rwm_body(const KernelArgs& a) {
    const StepArgs& s = a.s;
    const P p(s, true);
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    double x[P::NC], sc[P::NC];
    p.load(a.st.x, s.ld, x);                                    // in flight while the tables are staged
    double lp = p.load_scalar(a.st.lp);
    p.stage();
#pragma unroll
    for (int k = 0; k < P::NC; ++k) sc[k] = p.valid(k) ? (US ? s.scale1 : s.scale[p.coord(k)]) : 0.0;
    AcceptDraw<P> ad;

    Keeper keep(s);
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        double xp[P::NC];
        gen_normals(p, rs, chain, (uint32_t)i, xp);             // xp <- z
#pragma unroll
        for (int k = 0; k < P::NC; ++k) xp[k] = x[k] + xp[k] * sc[k];   // pars + randn(d) .* scale
        bool oos;
        const double lpp = eval_lp(p, model, xp, oos);
        const double ratio = lpp - lp;
        const bool acc = ad.test(p, rs, chain, i, t, ratio);
        if (acc) {
#pragma unroll
            for (int k = 0; k < P::NC; ++k) x[k] = xp[k];
            lp = lpp;
        }
        int64_t kk;
        if (keep.take(i, &kk)) {
            p.store_kept(s, kk, x, s.samples);
            p.store_bit(s, kk, acc);
        }
    }
    p.store(a.st.x, s.ld, x);
    p.store_t(a.st.lp, lp);
    p.count_evals(s, s.nsteps);
}

// ------------------------------------------------------------------ MALA
template <class P, class M>
__device__ __forceinline__ void mala_body(const KernelArgs& a) {
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const P p(s);
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    double x[P::NC];
    p.load(a.st.x, s.ld, x);
    double lp = p.load_scalar(a.st.lp);
    double h = sa.tuner ? p.load_scalar(a.st.t_step) : sa.drift_step;
    int32_t n_acc = sa.tuner ? p.load_t(a.st.t_acc) : 0;
    int32_t n_prop = sa.tuner ? p.load_t(a.st.t_prop) : 0;
    AcceptDraw<P> ad;

    Keeper keep(s);
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        if (sa.tuner) n_prop += 1;
        const double half = h / 2.0;
        const double sq = __builtin_sqrt(h);
        const double twoh = 2.0 * h;
        const double L = det_log(kTwoPi * h) / 2.0;             // log(2*pi*driftStep)/2
        double xp[P::NC];
        gen_normals(p, rs, chain, (uint32_t)i, xp);
        double qf = 0.0;
        const GradAt<M, P::NC> gx(model, x);
#pragma unroll
        for (int k = 0; k < P::NC; ++k) {
            const double pm = x[k] + half * gx(k, x[k]);        // parsMean (MALA.jl:98)
            xp[k] = pm + sq * xp[k];                            // MALA.jl:100
            const double e = pm - xp[k];
            if (p.valid(k)) qf = qf + ((-(e * e)) / twoh - L);  // MALA.jl:103
        }
        qf = p.reduce(qf);
        bool oos;
        const double lpp = eval_lp(p, model, xp, oos);
        double qb = 0.0;
        const GradAt<M, P::NC> gxp(model, xp, !oos);
#pragma unroll
        for (int k = 0; k < P::NC; ++k) {
            const double gp = oos ? 0.0 : gxp(k, xp[k]);
            const double e = (xp[k] + half * gp) - x[k];       // MALA.jl:104-105
            if (p.valid(k)) qb = qb + ((-(e * e)) / twoh - L);
        }
        qb = p.reduce(qb);
        const double ratio = ((lpp + qb) - lp) - qf;            // MALA.jl:107
        const bool acc = ad.test(p, rs, chain, i, t, ratio);
        if (acc) {
#pragma unroll
            for (int k = 0; k < P::NC; ++k) x[k] = xp[k];
            lp = lpp;
            if (sa.tuner) n_acc += 1;
        }
        int64_t kk;
        if (keep.take(i, &kk)) {
            p.store_kept(s, kk, x, s.samples);
            if (s.grads != nullptr) {
                double g[P::NC];
                const GradAt<M, P::NC> gk(model, x);
#pragma unroll
                for (int k = 0; k < P::NC; ++k) g[k] = gk(k, x[k]);
                p.store_kept(s, kk, g, s.grads);
            }
            p.store_bit(s, kk, acc);
        }
        if (sa.tuner && i <= s.tuner_burnin && (i % sa.adapt_step) == 0) {   // MALA.jl:116-118
            h = h * tune_factor(n_acc, n_prop, sa.target_rate);
            n_acc = 0;
            n_prop = 0;
        }
    }
    p.store(a.st.x, s.ld, x);
    p.store_t(a.st.lp, lp);
    p.count_evals(s, s.nsteps);
    if (sa.tuner) {
        p.store_t(a.st.t_step, h);
        p.store_t(a.st.t_acc, n_acc);
        p.store_t(a.st.t_prop, n_prop);
    }
}

// ------------------------------------------------------------------ HMC / HMCDA
// nl leapfrogs from (x, m) (HMC.jl:93-102); the start point is in support.
// Two restructurings, both bitwise neutral:
//  * the half kick (0.5 g) eps at a point is computed once and used by the closing half kick of one
//    leapfrog and the opening one of the next (the same x, the same oos flag) -- when the chain's
//    coordinates are few enough (NC <= 16) for the carried kicks to stay in registers;
//  * a model without the LLAcc rule (a function model) never goes out of support, so only the last
//    leapfrog's log-target is used: it is evaluated once, after the loop.
template <class P, class M>
__device__ __forceinline__ double trajectory(const P& p, const M& model, double eps, int64_t nl, double (&x)[P::NC],
                                             double (&m)[P::NC]) {
    constexpr bool kCarry = P::NC <= 16;
    // the uncarried branch reads model.grad per coordinate, which a joint model does not define (GradAt does)
    static_assert(kCarry || !is_joint<M>::value, "joint models run lane per chain (NC <= 16)");
    bool oos = false;
    double lpl = 0.0;
    double kick[kCarry ? P::NC : 1];
    if constexpr (kCarry) {
        const GradAt<M, P::NC> g0(model, x);
#pragma unroll
        for (int k = 0; k < P::NC; ++k) kick[k] = (0.5 * g0(k, x[k])) * eps;
    }
    for (int64_t l = 0; l < nl; ++l) {
#pragma unroll
        for (int k = 0; k < P::NC; ++k) {
            double a;
            if constexpr (kCarry) a = kick[k];
            else a = (0.5 * (oos ? 0.0 : model.grad(x[k]))) * eps;
            m[k] = m[k] + a;                                    // n.m += 0.5*n.grad*ve
            x[k] = x[k] + eps * m[k];                           // n.pars += ve * n.m
        }
        if (M::kLLAcc) lpl = eval_lp(p, model, x, oos);         // calc!(n, ll)
        const GradAt<M, P::NC> gl(model, x, !oos);
#pragma unroll
        for (int k = 0; k < P::NC; ++k) {
            const double g = oos ? 0.0 : gl(k, x[k]);
            const double a = (0.5 * g) * eps;
            if constexpr (kCarry) kick[k] = a;
            m[k] = m[k] + a;
        }
    }
    if (!M::kLLAcc && nl > 0) lpl = eval_lp(p, model, x, oos);
    return lpl;
}

// The same trajectory for a model whose half gradient 0.5 * (-2 x) is -x (IsoDot): the half kick is (-x) eps, one
// multiply instead of three, and bitwise trajectory()'s whenever |x| < 2^1023 (then -2x cannot overflow and
// the halving is exact, subnormals included).  big reports an |x| >= 2^1023 (or non-finite) anywhere on the
// path, where -2x would have overflowed: the caller then redoes the trajectory with trajectory().
template <class P, class M>
__device__ __forceinline__ double trajectory_halfneg(const P& p, const M& model, double eps, int64_t nl,
                                                     double (&x)[P::NC], double (&m)[P::NC], bool& big) {
    double kick[P::NC];
    double xmax = 0.0;
#pragma unroll
    for (int k = 0; k < P::NC; ++k) {
        kick[k] = (-x[k]) * eps;
        xmax = __builtin_fmax(xmax, __builtin_fabs(x[k]));
    }
    for (int64_t l = 0; l < nl; ++l) {
#pragma unroll
        for (int k = 0; k < P::NC; ++k) {
            m[k] = m[k] + kick[k];                                  // n.m += 0.5*n.grad*ve
            x[k] = x[k] + eps * m[k];                               // n.pars += ve * n.m
            kick[k] = (-x[k]) * eps;                                // 0.5*n.grad*ve at the new point
            xmax = __builtin_fmax(xmax, __builtin_fabs(x[k]));
            m[k] = m[k] + kick[k];                                  // n.m += 0.5*n.grad*ve
        }
    }
    big = p.any(!(xmax < 0x1p1023) && p.live);
    double lpl = 0.0;
    bool oos;
    if (nl > 0) lpl = eval_lp(p, model, x, oos);                    // calc!(n, ll) of the last leapfrog
    return lpl;
}

template <class P, class M, bool DA>
__device__ __forceinline__ void hmc_body(const KernelArgs& a) {
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const P p(s);
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    const int64_t max_leaps = sa.max_leaps;
    const bool tuned = !DA && sa.tuner;

    double x0[P::NC];
    p.load(a.st.x, s.ld, x0);
    double lp = p.load_scalar(a.st.lp);
    double eps = (DA || tuned) ? p.load_scalar(a.st.t_step) : sa.leap_step;
    int64_t nl_fixed = tuned ? (int64_t)p.load_t(a.st.t_leaps) : sa.n_leaps;
    double eps_bar = DA ? p.load_scalar(a.st.t_bar) : 0.0;
    double h_bar = DA ? p.load_scalar(a.st.t_h) : 0.0;
    int32_t n_acc = tuned ? p.load_t(a.st.t_acc) : 0;
    int32_t n_prop = tuned ? p.load_t(a.st.t_prop) : 0;
    const double mu = DA ? det_log(10.0) : 0.0;                 // log(10*leapStep0), leapStep0 = 1

    int64_t n_evals = 0;
    Keeper keep(s);
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        if (tuned) n_prop += 1;
        double m[P::NC], x[P::NC];
        gen_normals(p, rs, chain, (uint32_t)i, m);              // state0.m = randn(model.size)
        const double H0 = -lp + half_dot(p, m);                 // update!(state0)
#pragma unroll
        for (int k = 0; k < P::NC; ++k) x[k] = x0[k];
        int64_t nl;
        if (DA) {
            const double r = round_away(sa.len / eps);          // HMCDA.jl:104
            nl = r < 1.0 ? 1 : (r > (double)max_leaps ? max_leaps : (int64_t)r);
        } else {
            nl = nl_fixed;
        }
        n_evals += nl;
        double lpl;
        if constexpr (M::kHalfGradNeg) {
            bool big;
            lpl = trajectory_halfneg(p, model, eps, nl, x, m, big);
            if (big) {                                          // -2x overflowed somewhere: the exact path
                // the same draw again, from a step index the compiler cannot see is i: otherwise it reuses the first
                // draw's values and keeps them live across the trajectory (d = 1024 HMC: 214 -> 286 VGPRs)
                uint32_t si = (uint32_t)i;
                asm volatile("" : "+s"(si));
#pragma unroll
                for (int k = 0; k < P::NC; ++k) x[k] = x0[k];
                gen_normals(p, rs, chain, si, m);
                lpl = trajectory(p, model, eps, nl, x, m);
            }
        } else {
            lpl = trajectory(p, model, eps, nl, x, m);
        }
        const double H = -lpl + half_dot(p, m);
        const u32x4 w = rs.block(chain, (uint32_t)i, 0u, TAG_ACCEPT);
        const double u = uniform52(w.x, w.y);
        bool acc;
        double pa = 0.0;
        if (DA) {
            pa = __builtin_fmin(1.0, det_exp(H0 - H));          // HMCDA.jl:120 (Julia 0.2 min: NaN-ignoring)
            acc = u < pa;
        } else {
            acc = u < det_exp(H0 - H);                          // HMC.jl:154
        }
        if (acc) {
#pragma unroll
            for (int k = 0; k < P::NC; ++k) x0[k] = x[k];
            lp = lpl;
            if (tuned) n_acc += 1;
        }
        int64_t kk;
        if (keep.take(i, &kk)) {
            p.store_kept(s, kk, x0, s.samples);
            if (s.grads != nullptr) {
                double g[P::NC];
                const GradAt<M, P::NC> gk(model, x0);
#pragma unroll
                for (int k = 0; k < P::NC; ++k) g[k] = gk(k, x0[k]);
                p.store_kept(s, kk, g, s.grads);
            }
            p.store_bit(s, kk, acc);
        }
        if (DA) {
            const double di = (double)i;
            if (di < (double)s.tuner_burnin) {                  // HMCDA.jl:133-138
                double eta = 1.0 / (di + sa.t0);
                h_bar = (1.0 - eta) * h_bar + eta * (sa.rate - pa);
                eps = det_exp(mu - (__builtin_sqrt(di) * h_bar) / sa.shrinkage);
                eta = det_exp(det_log(di) * (-sa.step));        // i^(-step)
                eps_bar = det_exp((1.0 - eta) * det_log(eps_bar) + eta * det_log(eps));
            } else {
                eps = eps_bar;                                  // HMCDA.jl:140
            }
        } else if (tuned && i <= s.tuner_burnin && (i % sa.adapt_step) == 0) {   // HMC.jl:167-169
            eps = eps * tune_factor(n_acc, n_prop, sa.target_rate);
            double nlf = __builtin_ceil(sa.target_path / eps);
            if (nlf > (double)sa.max_step) nlf = (double)sa.max_step;
            if (nlf > (double)max_leaps) nlf = (double)max_leaps;
            nl_fixed = (int64_t)nlf;
            n_acc = 0;
            n_prop = 0;
        }
    }
    p.count_evals(s, n_evals);
    p.store(a.st.x, s.ld, x0);
    p.store_t(a.st.lp, lp);
    if (DA || tuned) p.store_t(a.st.t_step, eps);
    if (DA) {
        p.store_t(a.st.t_bar, eps_bar);
        p.store_t(a.st.t_h, h_bar);
    } else if (tuned) {
        p.store_t(a.st.t_leaps, (int32_t)nl_fixed);
        p.store_t(a.st.t_acc, n_acc);
        p.store_t(a.st.t_prop, n_prop);
    }
}

// ------------------------------------------------------------------ HMC storeLeaps (HMC.jl:145-150, HMCDA.jl:110-117)
// Records the trajectory the next step (s.step_begin) takes, without moving the chain: leap 0 is state0 after
// update! (pars, grad, momentum, logTarget, H), leap l the state after the l-th leapfrog (HMC.jl:93-102), for
// l <= min(nLeaps, cap); nl gets nLeaps.  hmc_body's and trajectory's operations, so the states are bitwise
// the ones the step computes; the log-target is evaluated after every leapfrog here (the step skips that for
// function models, where it does not feed back into the trajectory).
template <class P, class M, bool DA>
__device__ __forceinline__ void hmc_record_body(const KernelArgs& a, const LeapRec& r) {
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const P p(s);
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    const bool tuned = !DA && sa.tuner;
    const int64_t i = s.step_begin;
    double x[P::NC], m[P::NC], g[P::NC];
    p.load(a.st.x, s.ld, x);
    const double lp = p.load_scalar(a.st.lp);
    const double eps = (DA || tuned) ? p.load_scalar(a.st.t_step) : sa.leap_step;
    int64_t nl;
    if (DA) {
        const double rr = round_away(sa.len / eps);                  // HMCDA.jl:104
        nl = rr < 1.0 ? 1 : (rr > (double)sa.max_leaps ? sa.max_leaps : (int64_t)rr);
    } else {
        nl = tuned ? (int64_t)p.load_t(a.st.t_leaps) : sa.n_leaps;
    }
    gen_normals(p, rs, chain, (uint32_t)i, m);                       // state0.m = randn(model.size)
    double H = -lp + half_dot(p, m);                                 // update!(state0)
    {
        const GradAt<M, P::NC> g0(model, x);
#pragma unroll
        for (int k = 0; k < P::NC; ++k) g[k] = g0(k, x[k]);          // the state's gradient (in support)
    }
    const size_t C = (size_t)s.C;
    p.store_cm(s, 0, x, r.pars);                                     // leapStates[1] = deepcopy(state0)
    p.store_cm(s, 0, g, r.grads);
    p.store_cm(s, 0, m, r.mom);
    p.store_t(r.lp, lp);
    p.store_t(r.H, H);
    bool oos = false;
    const int64_t nrec = nl < r.cap ? nl : r.cap;
    for (int64_t l = 1; l <= nrec; ++l) {
#pragma unroll
        for (int k = 0; k < P::NC; ++k) {
            m[k] = m[k] + (0.5 * g[k]) * eps;                         // n.m += 0.5*n.grad*ve
            x[k] = x[k] + eps * m[k];                                 // n.pars += ve * n.m
        }
        const double lpl = eval_lp(p, model, x, oos);                // calc!(n, ll)
        const GradAt<M, P::NC> gl(model, x, !oos);
#pragma unroll
        for (int k = 0; k < P::NC; ++k) {
            g[k] = oos ? 0.0 : gl(k, x[k]);
            m[k] = m[k] + (0.5 * g[k]) * eps;                         // n.m += 0.5*n.grad*ve
        }
        H = -lpl + half_dot(p, m);                                    // update!(n)
        p.store_cm(s, l, x, r.pars);                                  // leapStates[l+1]
        p.store_cm(s, l, g, r.grads);
        p.store_cm(s, l, m, r.mom);
        p.store_t(r.lp + (size_t)l * C, lpl);
        p.store_t(r.H + (size_t)l * C, H);
    }
    p.store_t(r.nl, (int32_t)nl);
}

// ------------------------------------------------------------------ RAM
// Robust adaptive Metropolis (RAM.jl:41-79), lane per chain.  x' = x + S z, RWM accept, then the
// jump factor S (packed rows in HBM, ram.hpp) takes the rank-1 update of RAM.jl:74-78.
template <class P, class M>
__device__ __forceinline__ void ram_body(const KernelArgs& a) {
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const P p(s);
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)p.c;
    constexpr int NC = P::NC;
    double x[NC];
    p.load(a.st.x, s.ld, x);
    double lp = p.load_scalar(a.st.lp);
    // the wave's 64-chain tile of each half of the factor store (ram.hpp), as buffer resources
    const uint64_t ld = (uint64_t)a.st.ram_ld;
    const uint32_t tile = (uint32_t)blockIdx.x * (kBlock / 64) + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double* const T0 = a.st.ram_L + (uint64_t)tile * (uint64_t)ram_tile_doubles(NC);
    const uint32_t vo = (threadIdx.x & 63) * 8;
    // rvec = randn(d) of step i and its S * rvec: the launch's first step forms them here, every later one
    // inside the previous step's factor update (ram_update<NEXT = true>), so a step reads the factor once.
    // kZLds (d > 4): the next rvec is drawn before the update into the lane's LDS slots and read back inside it:
    // the Box-Muller radius's rare-tail branches inside the fully unrolled factor sweep made it spill (800+ VGPRs at
    // d = 32).  8 KB a Philox block beside the 56 KB tables: two 256-thread blocks a CU up to d = 12, one beyond.
    constexpr bool kZLds = P::NB > 1;
    double* zlds = nullptr;
    if constexpr (kZLds) {
        __shared__ double zbuf[4 * P::NB * kBlock];
        zlds = zbuf;
    }
    double u[NC], nz = 0.0;
    if (s.nsteps > 0) {
        const int64_t i = s.step_begin;
        double z[NC];
        gen_normals(p, rs, chain, (uint32_t)i, z);
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (!p.valid(k)) z[k] = 0.0;                                    // padding: identity block
            nz = __builtin_fma(z[k], z[k], nz);                             // dot(rvec, rvec)
        }
        ram_matvec<NC>(ram_tile_rsrc<NC>(ram_half<NC>(T0, i - 1, ld)), vo, z, u);
    }
    Keeper keep(s);
    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        double lpp;
        {
            double xp[NC];
#pragma unroll
            for (int k = 0; k < NC; ++k) xp[k] = x[k] + u[k];                 // RAM.jl:60
            bool oos;
            lpp = eval_lp(p, model, xp, oos);
        }
        const double ratio = lpp - lp;
        const bool acc = mh_accept_short_circuit(rs, chain, (uint32_t)i, ratio);
        if (acc) {
            // the proposal is recomputed (bitwise the same sums) rather than held across the evaluation
#pragma unroll
            for (int k = 0; k < NC; ++k) x[k] = x[k] + u[k];
            lp = lpp;
        }
        int64_t kk;
        if (keep.take(i, &kk)) {
            p.store_kept(s, kk, x, s.samples);
            p.store_bit(s, kk, acc);
        }
        const double alpha = ram_alpha(i, s.d, ratio, sa.rate);
        const ram_rsrc_t Ss = ram_tile_rsrc<NC>(ram_half<NC>(T0, i - 1, ld));
        const ram_rsrc_t Sd = ram_tile_rsrc<NC>(ram_half<NC>(T0, i, ld));
        double un[NC], nzn = 0.0;
        auto zgen = [&](int b, double (&z4)[4]) {                             // step i + 1's rvec, block b
            const u32x4 w = rs.block(chain, (uint32_t)(i + 1), p.block(b), TAG_NORMAL);
            normals4(w, z4[0], z4[1], z4[2], z4[3], p.bt.rad, p.bt.sct);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!p.valid(4 * b + e)) z4[e] = 0.0;
                nzn = __builtin_fma(z4[e], z4[e], nzn);
            }
        };
        auto zblock = [&](int b, double (&z4)[4]) {
            if constexpr (kZLds) {                                            // drawn before the update
#pragma unroll
                for (int e = 0; e < 4; ++e) z4[e] = zlds[(4 * b + e) * kBlock + threadIdx.x];
            } else {
                zgen(b, z4);
            }
        };
        if (kZLds && t + 1 < s.nsteps) {
#pragma unroll
            for (int b = 0; b < P::NB; ++b) {
                double z4[4];
                zgen(b, z4);
#pragma unroll
                for (int e = 0; e < 4; ++e) zlds[(4 * b + e) * kBlock + threadIdx.x] = z4[e];
            }
        }
        if (t + 1 < s.nsteps) {
            ram_update<NC, true>(Ss, Sd, vo, alpha, nz, u, zblock, un);
#pragma unroll
            for (int k = 0; k < NC; ++k) u[k] = un[k];
            nz = nzn;
        } else {
            ram_update<NC, false>(Ss, Sd, vo, alpha, nz, u, zblock, un);
        }
    }
    p.store(a.st.x, s.ld, x);
    p.store_t(a.st.lp, lp);
    p.count_evals(s, s.nsteps);
}

// ------------------------------------------------------------------ eval
// lp (and gradient) of x; flags out-of-support starts (RWM.jl:54-55).
template <class P, class M>
__device__ __forceinline__ void eval_body(const KernelArgs& a, const double* xin, double* lp_out, double* g_out,
                                          int32_t check) {
    const StepArgs& s = a.s;
    const P p(s);
    const M model(a.m);
    double x[P::NC];
    p.load(xin, s.ld, x);
    bool oos;
    const double lp = eval_lp(p, model, x, oos);
    p.store_t(lp_out, lp);
    if (g_out != nullptr) {
        double g[P::NC];
        const GradAt<M, P::NC> gx(model, x, !oos);
#pragma unroll
        for (int k = 0; k < P::NC; ++k) g[k] = oos ? 0.0 : gx(k, x[k]);
        p.store(g_out, s.ld, g);
    }
    if (check && p.live && !(lp - lp == 0.0)) atomicOr(s.err, 1);
}

}  // namespace mcmc
