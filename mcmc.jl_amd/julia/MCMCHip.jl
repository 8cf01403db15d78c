# MCMCHip.jl -- Julia binding of include/mcmc_hip.h (text only: this image has no Julia; see INTEGRATION.md)
module MCMCHip
const lib = "libmcmc_hip"          # on LD_LIBRARY_PATH, or an absolute path to mcmchip/libmcmc_hip.so

# ---- structs: field order and types mirror include/mcmc_hip.h exactly (isbits, C layout)
struct ModelDesc                   # mcmc_model_desc
    kind::Int32; has_gradient::Int32; d::Int64
    init::Ptr{Float64}; scale::Ptr{Float64}
    mu::Float64; sigma::Float64; prior_sigma::Float64; noise_sigma::Float64; link_sign::Float64
    n::Int64; X::Ptr{Float64}; Y::Ptr{Float64}
    dist::Int32                    # MODEL_DIST_DSL: MCMC_DIST_*, parameters in mu / sigma
end
struct SamplerCfg                  # mcmc_sampler_cfg
    kind::Int32; scale::Float64; drift_step::Float64; n_leaps::Int64; leap_step::Float64
    rate::Float64; len::Float64; shrinkage::Float64; t0::Float64; step::Float64
    tuner::Int32; adapt_step::Int64; max_step::Int64; target_path::Float64; target_rate::Float64
    max_leaps::Int64
end
struct RunnerCfg; burnin::Int64; thinning::Int64; len::Int64; end
mutable struct Outputs             # mcmc_outputs (mutable: the library writes runtime_s, kernel_ms, nkept)
    samples::Ptr{Float64}; gradients::Ptr{Float64}; accept_bits::Ptr{UInt64}
    final_x::Ptr{Float64}; final_lp::Ptr{Float64}; on_device::Int32
    runtime_s::Float64; kernel_ms::Float64; nkept::Int64
end

const MODEL_ISO_NORMAL_DOT, MODEL_NORMAL_DSL, MODEL_LOGISTIC, MODEL_LINEAR = 1, 2, 3, 4
const MODEL_ABS_NORMAL_DSL, MODEL_DIST_DSL, MODEL_PROBIT, MODEL_DIST_OBS, MODEL_OU = 5, 6, 7, 8, 9
const RWM_K, MALA_K, HMC_K, HMCDA_K, RAM_K = 1, 2, 3, 4, 5

check(st) = st == 0 ? nothing :
    error(unsafe_string(ccall((:mcmc_last_error, lib), Cstring, ())))   # reference @assert text

function context(device::Integer = 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:mcmc_ctx_create, lib), Cint, (Cint, Ptr{Ptr{Cvoid}}), device, h))
    h[]
end

# model(v -> -dot(v,v), grad = v -> -2v, init = ...)   (README.md:60-63)
function isonormal_model(ctx, init::Vector{Float64}; scale = ones(length(init)))
    desc = ModelDesc(MODEL_ISO_NORMAL_DOT, 1, length(init), pointer(init), pointer(scale),
                     0.0, 1.0, 1.0, 1.0, 1.0, 0, C_NULL, C_NULL, 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve init scale check(ccall((:mcmc_model_create, lib), Cint,
        (Ptr{Cvoid}, Ref{ModelDesc}, Ptr{Ptr{Cvoid}}), ctx, desc, h))
    h[]
end

# examples/logistic_regression.jl:16-22: X is n x d; the ABI wants row-major [n][d] = Julia X' (column-major)
function logistic_model(ctx, X::Matrix{Float64}, Y::Vector{Float64}; init = zeros(size(X, 2)))
    Xr = collect(transpose(X)); scale = ones(size(X, 2))
    desc = ModelDesc(MODEL_LOGISTIC, 1, size(X, 2), pointer(init), pointer(scale),
                     0.0, 1.0, 1.0, 1.0, 1.0, size(X, 1), pointer(Xr), pointer(Y), 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve Xr Y init scale check(ccall((:mcmc_model_create, lib), Cint,
        (Ptr{Cvoid}, Ref{ModelDesc}, Ptr{Ptr{Cvoid}}), ctx, desc, h))
    h[]
end

# examples/ornstein.jl:19-30: the series x (passed as Y), parameters (tau, sigma, mu) from the example's start and
# scale hint (ornstein.jl:29-30)
function ou_model(ctx, x::Vector{Float64}; init = [0.05, 1.0, 1.0], scale = [1000.0, 1.0, 10.0])
    desc = ModelDesc(MODEL_OU, 1, 3, pointer(init), pointer(scale), 0.0, 1.0, 1.0, 1.0, 1.0, length(x), C_NULL,
                     pointer(x), 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve x init scale check(ccall((:mcmc_model_create, lib), Cint,
        (Ptr{Cvoid}, Ref{ModelDesc}, Ptr{Ptr{Cvoid}}), ctx, desc, h))
    h[]
end

rwm(scale) = SamplerCfg(RWM_K, scale, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
hmc(n, eps) = SamplerCfg(HMC_K, 0, 0, n, eps, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
hmcda(; rate=0.65, len=2., shrinkage=0.05, t0=10., step=0.75) =
    SamplerCfg(HMCDA_K, 0, 0, 0, 0, rate, len, shrinkage, t0, step, 0, 0, 0, 0, 0, 0)
ram(scale = 1.0, rate = 0.234) = SamplerCfg(RAM_K, scale, 0, 0, 0, rate, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)   # RAM.jl:22-34

function chains(model, s::SamplerCfg, nchains; seed = 1, offset = 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:mcmc_chains_create, lib), Cint,
        (Ptr{Cvoid}, Ref{SamplerCfg}, Int64, Int64, UInt64, Ptr{Float64}, Ptr{Ptr{Cvoid}}),
        model, s, nchains, offset, seed, C_NULL, h))
    h[]
end

# MCMC.reset(t, x) (MCMC.jl:39): every chain at x (d x C) with its log-target re-evaluated there; returns the lp
function reset!(ch, x::Matrix{Float64})
    lp = Vector{Float64}(undef, size(x, 2))
    xt = collect(transpose(x))                                   # [d][C] in C order = Julia (C, d)
    GC.@preserve xt lp check(ccall((:mcmc_chains_set_state, lib), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}),
                                   ch, xt, lp))
    lp
end

# chains first+1 .. first+count of ch as an independent batch that continues them (mcmc_chains_fork)
function fork(ch, first::Integer, count::Integer)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:mcmc_chains_fork, lib), Cint, (Ptr{Cvoid}, Int64, Int64, Ptr{Ptr{Cvoid}}), ch, first, count, h))
    h[]
end

# optional: size the library's staging buffers once, so that timed runs allocate nothing
reserve(ch, nkept; on_device = false) =
    check(ccall((:mcmc_chains_reserve_outputs, lib), Cint, (Ptr{Cvoid}, Int64, Int32), ch, nkept, on_device))

# run_serialmc (SerialMC.jl:37-85): returns samples[nkept][d][C] (Julia: Array{Float64,3} of size (C, d, nkept))
function run_serialmc(ch, d, C; steps, burnin = 0, thinning = 1)
    r = (burnin+1):thinning:steps
    smp = Array{Float64}(undef, C, d, length(r))
    bits = zeros(UInt64, cld(C, 64), length(r))
    out = Outputs(pointer(smp), C_NULL, pointer(bits), C_NULL, C_NULL, 0, 0.0, 0.0, 0)
    GC.@preserve smp bits check(ccall((:mcmc_run_serialmc, lib), Cint,
        (Ptr{Cvoid}, Ref{RunnerCfg}, Ref{Outputs}), ch, RunnerCfg(burnin, thinning, steps), out))
    accept = [(bits[fld(c, 64) + 1, j] >> (c % 64)) & 1 == 1 for c in 0:C-1, j in 1:length(r)]
    smp, accept, out.runtime_s
end

# ---- prun (runners.jl:35-42, examples/parallel_serialmc.jl) -> one chain batch over a node's GPUs
# mcmc_group_*: contiguous 64-chain-aligned blocks, one per listed device, driven from this one Julia thread
# (a library worker thread per block); results bit-identical to one context running every chain.  Blocks are whole
# 64-chain groups, so a batch of fewer than 64 N chains leaves trailing devices idle.  The handles are freed by
# finalizers (or destroy! explicitly); a group whose chains are still alive is kept (the library refuses it) and released
# by the destroy! of its last GroupChains, whatever order the finalizers run in.
mutable struct Group
    h::Ptr{Cvoid}
    released::Bool                 # destroy! was called (explicitly or by the finalizer)
    function Group(h)
        g = new(h, false)
        finalizer(destroy!, g)
    end
end
mutable struct GroupChains
    h::Ptr{Cvoid}
    group::Group
    function GroupChains(h, g)
        gc = new(h, g)
        finalizer(destroy!, gc)
    end
end
function destroy!(gc::GroupChains)
    gc.h == C_NULL || ccall((:mcmc_group_chains_destroy, lib), Cint, (Ptr{Cvoid},), gc.h)
    gc.h = C_NULL
    # Julia does not order the finalizers of objects collected in one cycle: if the group's ran first, the library
    # refused it (chains alive) and the group kept its handle; with these chains gone, release it now
    gc.group.released && release_group!(gc.group)
    nothing
end
function release_group!(g::Group)
    g.h == C_NULL && return
    # refused while any GroupChains of the group is alive: keep the handle, the last one retries
    ccall((:mcmc_group_destroy, lib), Cint, (Ptr{Cvoid},), g.h) == 0 && (g.h = C_NULL)
    nothing
end
function destroy!(g::Group)
    g.released = true
    release_group!(g)
end

function device_count()
    n = Ref{Cint}(0)
    check(ccall((:mcmc_device_count, lib), Cint, (Ptr{Cint},), n))
    Int(n[])
end

# default: every visible device
function group(devices::Vector{Int32} = Int32.(0:device_count()-1))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:mcmc_group_create, lib), Cint, (Ptr{Int32}, Int32, Ptr{Ptr{Cvoid}}), devices, length(devices), h))
    Group(h[])
end

# the model descriptor is uploaded once per device; init/scale (and X/Y) must stay rooted during the call
function group_chains(g::Group, desc::ModelDesc, s::SamplerCfg, nchains; seed = 1, offset = 0, roots = ())
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve roots check(ccall((:mcmc_group_chains_create, lib), Cint,
        (Ptr{Cvoid}, Ref{ModelDesc}, Ref{SamplerCfg}, Int64, Int64, UInt64, Ptr{Float64}, Ptr{Ptr{Cvoid}}),
        g.h, desc, s, nchains, offset, seed, C_NULL, h))
    GroupChains(h[], g)
end

# every block's step loop concurrently, then each GPU's outputs device -> host into its columns of smp / bits
# (the library page-locks smp / bits for the call, so the gather is direct DMA)
function run_serialmc_group(gc::GroupChains, d, C; steps, burnin = 0, thinning = 1)
    r = (burnin+1):thinning:steps
    smp = Array{Float64}(undef, C, d, length(r))
    bits = zeros(UInt64, cld(C, 64), length(r))
    out = Outputs(pointer(smp), C_NULL, pointer(bits), C_NULL, C_NULL, 0, 0.0, 0.0, 0)
    gather = Ref{Float64}(0.0)
    GC.@preserve smp bits check(ccall((:mcmc_group_run_serialmc, lib), Cint,
        (Ptr{Cvoid}, Ref{RunnerCfg}, Ref{Outputs}, Ref{Float64}), gc.h, RunnerCfg(burnin, thinning, steps), out, gather))
    accept = [(bits[fld(c, 64) + 1, j] >> (c % 64)) & 1 == 1 for c in 0:C-1, j in 1:length(r)]
    smp, accept, out.runtime_s, gather[]
end
end # module
