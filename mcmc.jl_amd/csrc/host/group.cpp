// group.cpp -- one node's GPUs driven by one host thread (include/mcmc_hip.h, mcmc_group_*).
//
// The reference parallelises only by mapping independent tasks over worker processes (prun -> pmap,
// src/runners/runners.jl:35-42).  Here one chain batch is split into contiguous blocks of whole 64-chain
// groups, one block per listed device, each an ordinary mcmc_chains on its own context (model data
// replicated per context).  The random streams are keyed by global chain id, so any split reproduces the
// one-context run bit for bit.  A run starts one worker thread per block: each drives its block's step
// loop on its own stream (no collective, no host synchronisation between blocks inside the loop) and then
// copies the block's outputs device -> host straight into its columns of the caller's buffers -- the end
// gather, over each GPU's own host link, concurrently.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "internal.hpp"

struct mcmc_group {
    std::vector<int> devices;
    std::vector<mcmc_ctx*> ctx;      // one context (stream) per listed device, also for a repeated device
    int chains_alive = 0;
};

struct mcmc_group_chains {
    mcmc_group* group = nullptr;
    int64_t C = 0, d = 0;
    std::vector<int64_t> first, count;
    std::vector<mcmc_model*> model;  // per block (NULL for an empty block)
    std::vector<mcmc_chains*> chains;
    // a run in which some block failed leaves the blocks at different steps: every later run is refused
    // until mcmc_group_chains_reset puts all blocks back at model.init (the bit-identity with one context
    // would otherwise be lost silently)
    bool failed = false;
    std::string fail_msg;
    int32_t inject_fail = -1;        // mcmc_debug_group_inject_failure: this block's next run fails before it starts
    double last_pin_s = 0.0;         // the last run's page-locking of the caller's outputs (register + release)
};

static int bad(const char* msg) { return mcmc_set_error(MCMC_E_INVALID_ARG, msg); }

static int64_t kept_rows(const mcmc_runner_cfg& r) {        // length of (burnin+1):thinning:len
    return r.len <= r.burnin ? 0 : (r.len - r.burnin - 1) / r.thinning + 1;
}

extern "C" int mcmc_group_plan(int64_t nchains, int32_t nblocks, int64_t* first, int64_t* count) {
    if (nchains <= 0 || nblocks <= 0 || !first || !count) return bad("bad argument");
    const int64_t per = (nchains + nblocks - 1) / nblocks;
    const int64_t blk = (per + 63) / 64 * 64;                    // whole 64-chain groups (accept-bit words)
    for (int32_t g = 0; g < nblocks; ++g) {
        const int64_t lo = std::min(nchains, (int64_t)g * blk);
        first[g] = lo;
        count[g] = std::min(nchains, lo + blk) - lo;
    }
    return MCMC_OK;
}

extern "C" int mcmc_group_create(const int32_t* devices, int32_t ndevices, mcmc_group** out) {
    if (!devices || ndevices <= 0 || !out) return bad("bad argument");
    *out = nullptr;
    auto* g = new mcmc_group();
    for (int32_t i = 0; i < ndevices; ++i) {
        mcmc_ctx* c = nullptr;
        if (int rc = mcmc_ctx_create(devices[i], &c)) {
            for (mcmc_ctx* x : g->ctx) mcmc_ctx_destroy(x);
            delete g;
            return rc;                                           // message set by mcmc_ctx_create
        }
        g->devices.push_back(devices[i]);
        g->ctx.push_back(c);
    }
    *out = g;
    return MCMC_OK;
}

extern "C" int mcmc_group_destroy(mcmc_group* g) {
    if (!g) return MCMC_OK;
    if (g->chains_alive) return bad("mcmc_group_destroy: chains of this group are still alive");
    for (mcmc_ctx* c : g->ctx) mcmc_ctx_destroy(c);
    delete g;
    return MCMC_OK;
}

extern "C" int mcmc_group_size(mcmc_group* g, int32_t* n) {
    if (!g || !n) return bad("NULL argument");
    *n = (int32_t)g->ctx.size();
    return MCMC_OK;
}

static void free_blocks(mcmc_group_chains* gc) {
    for (mcmc_chains* c : gc->chains)
        if (c) mcmc_chains_destroy(c);
    for (mcmc_model* m : gc->model)
        if (m) mcmc_model_destroy(m);
    gc->chains.clear();
    gc->model.clear();
}

extern "C" int mcmc_group_chains_create(mcmc_group* g, const mcmc_model_desc* desc, const mcmc_sampler_cfg* s,
                                        int64_t nchains, int64_t chain_offset, uint64_t seed, const double* init_x,
                                        mcmc_group_chains** out) {
    if (!g || !desc || !s || !out) return bad("NULL argument");
    *out = nullptr;
    if (nchains <= 0) return bad("nchains should be > 0");
    const int32_t G = (int32_t)g->ctx.size();
    auto* gc = new mcmc_group_chains();
    gc->group = g;
    gc->C = nchains;
    gc->d = desc->d;
    gc->first.resize(G);
    gc->count.resize(G);
    gc->model.assign(G, nullptr);
    gc->chains.assign(G, nullptr);
    mcmc_group_plan(nchains, G, gc->first.data(), gc->count.data());
    std::vector<double> xi;
    for (int32_t b = 0; b < G; ++b) {
        if (gc->count[b] == 0) continue;
        int rc = mcmc_model_create(g->ctx[b], desc, &gc->model[b]);
        const double* bx = nullptr;
        if (rc == MCMC_OK && init_x) {                           // this block's columns of [d][nchains]
            const int64_t n = gc->count[b], f = gc->first[b];
            xi.resize((size_t)desc->d * n);
            for (int64_t j = 0; j < desc->d; ++j)
                std::copy(init_x + j * nchains + f, init_x + j * nchains + f + n, xi.begin() + j * n);
            bx = xi.data();
        }
        if (rc == MCMC_OK)
            rc = mcmc_chains_create(gc->model[b], s, gc->count[b], chain_offset + gc->first[b], seed, bx,
                                    &gc->chains[b]);
        if (rc != MCMC_OK) {
            const std::string msg = mcmc_last_error();
            free_blocks(gc);
            delete gc;
            return mcmc_set_error(rc, msg);
        }
    }
    g->chains_alive += 1;
    *out = gc;
    return MCMC_OK;
}

extern "C" int mcmc_group_chains_destroy(mcmc_group_chains* gc) {
    if (!gc) return MCMC_OK;
    free_blocks(gc);
    gc->group->chains_alive -= 1;
    delete gc;
    return MCMC_OK;
}

extern "C" int mcmc_group_chains_reset(mcmc_group_chains* gc) {
    if (!gc) return bad("NULL argument");
    for (mcmc_chains* c : gc->chains)
        if (c)
            if (int rc = mcmc_chains_reset(c)) return rc;       // still failed: a block kept its old state
    gc->failed = false;
    gc->fail_msg.clear();
    return MCMC_OK;
}

extern "C" int mcmc_group_chains_steps_done(mcmc_group_chains* gc, int64_t* steps) {
    if (!gc || !steps) return bad("NULL argument");
    int64_t s0 = -1;
    for (mcmc_chains* c : gc->chains) {
        if (!c) continue;
        int64_t s = 0;
        if (int rc = mcmc_chains_steps_done(c, &s)) return rc;
        if (s0 >= 0 && s != s0)
            return mcmc_set_error(MCMC_E_INVALID_ARG, "mcmc_group_chains_steps_done: the blocks are at different "
                                                      "steps (a failed run); mcmc_group_chains_reset first");
        s0 = s;
    }
    if (s0 < 0) return bad("no chains");
    *steps = s0;
    return MCMC_OK;
}

extern "C" int mcmc_group_chains_set_steps_per_launch(mcmc_group_chains* gc, int64_t spl) {
    if (!gc) return bad("NULL argument");
    for (mcmc_chains* c : gc->chains)
        if (c)
            if (int rc = mcmc_chains_set_steps_per_launch(c, spl)) return rc;
    return MCMC_OK;
}

extern "C" int mcmc_group_chains_block(mcmc_group_chains* gc, int32_t b, mcmc_chains** chains, int64_t* first,
                                       int64_t* count) {
    if (!gc || b < 0 || b >= (int32_t)gc->chains.size()) return bad("bad block index");
    if (chains) *chains = gc->chains[b];
    if (first) *first = gc->first[b];
    if (count) *count = gc->count[b];
    return MCMC_OK;
}

// The caller's host output buffers, page-locked for the gather: a buffer that is not already pinned is
// registered (portable: visible to every device's copy engine) for the duration of the run and released after
// it.  Device -> host copies into pageable memory are staged through a driver bounce buffer at a fraction of
// the link rate; into pinned memory they are direct DMA.
// reg_s: the registration plus (release()) the unregistration time, reported apart from the copies
// (mcmc_group_last_pin_s): at the metric size it is comparable to the gather itself.
struct PinnedOutputs {
    std::vector<void*> registered;
    double reg_s = 0.0;
    void pin(void* p, size_t bytes) {
        if (!p || bytes == 0) return;
        const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
        if (e == hipSuccess) registered.push_back(p);
        else (void)hipGetLastError();           // already pinned (hipErrorHostMemoryAlreadyRegistered) or not
                                                // registrable: the copy still works, staged
    }
    void release() {
        const auto c0 = std::chrono::steady_clock::now();
        for (void* p : registered) (void)hipHostUnregister(p);
        registered.clear();
        reg_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
    }
    ~PinnedOutputs() { release(); }
};

extern "C" int mcmc_group_run_serialmc(mcmc_group_chains* gc, const mcmc_runner_cfg* r, mcmc_outputs* out,
                                       double* gather_s) {
    if (!gc || !r) return bad("NULL argument");
    if (int rc = mcmc_runner_validate(r)) return rc;
    if (out && out->on_device) return bad("group runs write host buffers (on_device must be 0)");
    if (gc->failed)
        return mcmc_set_error(MCMC_E_INVALID_ARG, "mcmc_group_run_serialmc: an earlier run of these chains failed (" +
                                                      gc->fail_msg + "); mcmc_group_chains_reset first");
    const int32_t G = (int32_t)gc->chains.size();
    const int64_t C = gc->C;
    struct Res {
        int rc = MCMC_OK;
        std::string msg;
        mcmc_outputs o{};
        double copy_s = 0.0;
    };
    std::vector<Res> res(G);
    PinnedOutputs pins;
    if (out) {
        const size_t nk = (size_t)kept_rows(*r), d = (size_t)gc->d, nw = (size_t)(C + 63) / 64;
        auto c0 = std::chrono::steady_clock::now();
        pins.pin(out->samples, nk * d * (size_t)C * 8);
        pins.pin(out->gradients, nk * d * (size_t)C * 8);
        pins.pin(out->accept_bits, nk * nw * 8);
        pins.pin(out->final_x, d * (size_t)C * 8);
        pins.pin(out->final_lp, (size_t)C * 8);
        pins.reg_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
    }
    auto work = [&](int32_t b) {
        Res& R = res[b];
        mcmc_outputs* po = nullptr;
        if (out) {                                               // this block's columns of the caller's buffers
            const int64_t f = gc->first[b];
            R.o.samples = out->samples ? out->samples + f : nullptr;
            R.o.gradients = out->gradients ? out->gradients + f : nullptr;
            R.o.accept_bits = out->accept_bits ? out->accept_bits + f / 64 : nullptr;
            R.o.final_x = out->final_x ? out->final_x + f : nullptr;
            R.o.final_lp = out->final_lp ? out->final_lp + f : nullptr;
            R.o.on_device = 0;
            po = &R.o;
        }
        if (b == gc->inject_fail) {
            R.rc = MCMC_E_HIP;
            R.msg = "injected failure (mcmc_debug_group_inject_failure)";
            return;
        }
        R.rc = mcmc_run_serialmc_ld(gc->chains[b], r, po, C, &R.copy_s);
        if (R.rc) R.msg = mcmc_last_error();                     // the worker's thread-local message
    };
    std::vector<int32_t> blocks;
    for (int32_t b = 0; b < G; ++b)
        if (gc->chains[b]) blocks.push_back(b);
    if (blocks.empty()) return bad("no chains");
    std::vector<std::thread> th;
    bool spawn_failed = false;
    try {
        for (size_t i = 0; i + 1 < blocks.size(); ++i) th.emplace_back(work, blocks[i]);
    } catch (...) {                                              // std::system_error: no thread could be started
        spawn_failed = true;
    }
    if (!spawn_failed) work(blocks.back());                      // the calling thread drives one block itself
    for (auto& t : th) t.join();                                 // every started worker, also after a failure
    gc->inject_fail = -1;
    if (spawn_failed) {
        // blocks whose worker started have advanced; the others have not
        gc->failed = true;
        gc->fail_msg = "could not start a worker thread";
        return mcmc_set_error(MCMC_E_HIP, "mcmc_group_run_serialmc: could not start a worker thread");
    }
    pins.release();
    gc->last_pin_s = pins.reg_s;
    double rt = 0.0, kms = 0.0, gs = 0.0;
    for (int32_t b : blocks) {
        if (res[b].rc) {
            const std::string msg = "block " + std::to_string(b) + " (device " +
                                    std::to_string(gc->group->devices[b]) + "): " + res[b].msg;
            gc->failed = true;
            gc->fail_msg = msg;
            return mcmc_set_error(res[b].rc, msg);
        }
        rt = std::max(rt, res[b].o.runtime_s);
        kms = std::max(kms, res[b].o.kernel_ms);
        gs = std::max(gs, res[b].copy_s);
    }
    if (out) {
        out->runtime_s = rt;
        out->kernel_ms = kms;
        out->nkept = res[blocks.back()].o.nkept;
    }
    if (gather_s) *gather_s = gs;
    return MCMC_OK;
}

extern "C" int mcmc_group_last_pin_s(const mcmc_group_chains* gc, double* pin_s) {
    if (!gc || !pin_s) return bad("NULL argument");
    *pin_s = gc->last_pin_s;
    return MCMC_OK;
}

extern "C" int mcmc_debug_group_inject_failure(mcmc_group_chains* gc, int32_t block) {
    if (!gc || block < 0 || block >= (int32_t)gc->chains.size()) return bad("bad block index");
    gc->inject_fail = block;
    return MCMC_OK;
}
