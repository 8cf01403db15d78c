// seqmc.hip -- the population bookkeeping of the SeqMC runner (src/runners/SeqMC.jl:43-122) on the
// device: importance-weight update, the resampling trigger var(W) < trigger, multinomial resampling
// (cumulative weights + one Philox uniform per particle + lower-bound search) and the per-step store.
// The mutation itself is the ordinary sampler kernel, one step of each target's chain batch
// (particle n = chain n of every target).
//
// Reductions use one fixed order that oracle/oracle.c orc_seqmc restates bit for bit: kSeqT = 256
// threads, thread k owns particles [k*chunk, min((k+1)*chunk, N)) (chunk = ceil(N/256)) and sums them
// left to right; the 256 partial sums are then added left to right by one thread.
#include "../common.hpp"
#include "../detmath.hpp"
#include "../host/kernels_api.hpp"

namespace mcmc {

constexpr int kSeqT = 256;
enum : uint32_t { TAG_RESAMPLE = 2u };

// logW[n] += ll0[n] - logtarget[n]; logtarget[n] = plogtarget[n]   (SeqMC.jl:70-71)
__global__ void k_seqmc_weights(int64_t N, double* logW, const double* ll0, double* logtarget,
                                const double* plogtarget) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    logW[n] = logW[n] + (ll0[n] - logtarget[n]);
    logtarget[n] = plogtarget[n];
}

// W = exp(logW); flag = var(W) < trigger (SeqMC.jl:76-77); cp = cumsum(W) / sum(W) (SeqMC.jl:78)
__global__ __launch_bounds__(kSeqT) void k_seqmc_scan(int64_t N, const double* logW, double trigger, double* cp,
                                                      int32_t* flag) {
    __shared__ double part[kSeqT];
    __shared__ double bcast[2];
    const int k = threadIdx.x;
    const int64_t chunk = (N + kSeqT - 1) / kSeqT;
    const int64_t b = (int64_t)k * chunk, e = b + chunk < N ? b + chunk : N;
    double s = 0.0;
    for (int64_t n = b; n < e; ++n) s = s + det_exp(logW[n]);
    part[k] = s;
    __syncthreads();
    if (k == 0) {
        double tot = 0.0;
        for (int i = 0; i < kSeqT; ++i) tot = tot + part[i];
        bcast[0] = tot;
    }
    __syncthreads();
    const double total = bcast[0];
    const double mean = total / (double)N;
    double q = 0.0;
    for (int64_t n = b; n < e; ++n) {
        const double dv = det_exp(logW[n]) - mean;
        q = q + dv * dv;
    }
    __syncthreads();                          // every thread has read bcast[0]; part[] is reused
    const double mine = s;
    part[k] = q;
    __syncthreads();
    if (k == 0) {
        double ss = 0.0;
        for (int i = 0; i < kSeqT; ++i) ss = ss + part[i];
        const double var = ss / (double)(N - 1);
        *flag = var < trigger ? 1 : 0;
    }
    __syncthreads();
    // exclusive scan of the chunk sums, left to right, then each chunk's running prefix
    part[k] = mine;
    __syncthreads();
    if (k == 0) {
        double run = 0.0;
        for (int i = 0; i < kSeqT; ++i) {
            const double v = part[i];
            part[i] = run;
            run = run + v;
        }
    }
    __syncthreads();
    double pre = part[k];
    for (int64_t n = b; n < e; ++n) {
        pre = pre + det_exp(logW[n]);
        cp[n] = pre / total;
    }
}

// resample (SeqMC.jl:79-87) when *flag: rs[n] = first p with cp[p] >= u_n, u_n one Philox uniform of
// (particle n, outer step, target index, TAG_RESAMPLE); pars_out[:, n] = pars[:, rs[n]],
// logtarget_out[n] = logtarget[rs[n]], logW[n] = 0.  Otherwise a copy.
__global__ void k_seqmc_resample(int64_t N, int d, const double* cp, const int32_t* flag, uint32_t key0,
                                 uint32_t key1, uint32_t step, uint32_t target, const double* pars,
                                 double* pars_out, const double* logtarget, double* logtarget_out, double* logW) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    int64_t src = n;
    if (*flag) {
        const u32x4 w = philox4x32_10((uint32_t)n, step, target, TAG_RESAMPLE, key0, key1);
        const double u = uniform52(w.x, w.y);
        int64_t lo = 0, hi = N - 1;                  // cp[N-1] == 1 > u: the search always succeeds
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo) / 2;
            if (cp[mid] >= u) hi = mid;
            else lo = mid + 1;
        }
        src = lo;
        logW[n] = 0.0;
    }
    for (int j = 0; j < d; ++j) pars_out[(size_t)j * N + n] = pars[(size_t)j * N + src];
    logtarget_out[n] = logtarget[src];
}

// store the particles and their weights exp(logW) of an outer step past burnin (SeqMC.jl:95-101)
__global__ void k_seqmc_store(int64_t N, int d, const double* pars, const double* logW, double* samples,
                              double* weights) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    for (int j = 0; j < d; ++j) samples[(size_t)j * N + n] = pars[(size_t)j * N + n];
    weights[n] = det_exp(logW[n]);
}

static unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace mcmc

hipError_t mcmc_seqmc_weights(int64_t N, double* logW, const double* ll0, double* logtarget, const double* plogtarget,
                              hipStream_t st) {
    mcmc::k_seqmc_weights<<<mcmc::nblk(N, 256), 256, 0, st>>>(N, logW, ll0, logtarget, plogtarget);
    return hipGetLastError();
}
hipError_t mcmc_seqmc_scan(int64_t N, const double* logW, double trigger, double* cp, int32_t* flag, hipStream_t st) {
    mcmc::k_seqmc_scan<<<1, mcmc::kSeqT, 0, st>>>(N, logW, trigger, cp, flag);
    return hipGetLastError();
}
hipError_t mcmc_seqmc_resample(int64_t N, int d, const double* cp, const int32_t* flag, uint64_t seed, uint32_t step,
                               uint32_t target, const double* pars, double* pars_out, const double* logtarget,
                               double* logtarget_out, double* logW, hipStream_t st) {
    mcmc::k_seqmc_resample<<<mcmc::nblk(N, 256), 256, 0, st>>>(N, d, cp, flag, (uint32_t)seed, (uint32_t)(seed >> 32),
                                                               step, target, pars, pars_out, logtarget, logtarget_out,
                                                               logW);
    return hipGetLastError();
}
hipError_t mcmc_seqmc_store(int64_t N, int d, const double* pars, const double* logW, double* samples, double* weights,
                            hipStream_t st) {
    mcmc::k_seqmc_store<<<mcmc::nblk(N, 256), 256, 0, st>>>(N, d, pars, logW, samples, weights);
    return hipGetLastError();
}
