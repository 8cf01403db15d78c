# mcmc_jl_hook.jl -- the MCMC.jl-side dispatch hook: `run(m * s * SerialMC(...))` on the GPU.
#
# Target: the Julia the reference package is written for (Julia 0.3 syntax: `immutable`/`type`, `Union(...)`,
# `{...}` Any-dicts, `Ptr{Void}`, `Uint8`, `finalizer(x, f)`, tasks with produce/consume).  It is include()d into
# module MCMC, after src/runners/SerialMC.jl (INTEGRATION.md §Julia hook shows the one line), so it sees MCMCModel,
# MCMCTask, MCMCChain, MCMCSample, HMCSample, SerialMC, RWM, MALA, HMC, HMCDA, RAM and EmpiricalMCMCTuner directly.
# For Julia >= 1.0 hosts without MCMC.jl, MCMCHip.jl is the plain binding of the same C ABI.
#
# What it replaces, with no edit to the reference's own files:
#   spinTask(m, s, r)           samplers.jl:53  -- a method for MCMCHipModel (more specific than MCMCModel): the task
#                                                  it returns produces MCMCSamples from a GPU chain instead of
#                                                  SamplerTask's CPU loop, so `m * s * r` (MCMC.jl:87-98), run(t)
#                                                  and run_serialmc (runners.jl:7-11, SerialMC.jl:37-85), run(c) (the
#                                                  continuation, runners.jl:14) and resume (SerialMC.jl:93-97) all
#                                                  run unchanged on top of it.  Each task installs the :reset hook
#                                                  (RWM.jl:49 ...) that MCMC.reset (MCMC.jl:39) and SeqMC
#                                                  (SeqMC.jl:68-69) call;
#   run(t::Array{MCMCTask})     runners.jl:17-33 -- redefined: tasks spun from one GPU model, sampler and runner (and
#                                                  not yet started) run as ONE chain batch, one mcmc_run_serialmc;
#                                                  each returned MCMCChain's task continues its own chain.  Any
#                                                  other array goes through the reference's dispatch as before;
#                                                  With SeqMC runners, GPU targets run as one mcmc_run_seqmc (one
#                                                  chain batch per target, a chain per particle) instead of
#                                                  run_seqmc's reset + consume per particle (SeqMC.jl:39-122);
#   prun(t::Array{MCMCTask})    runners.jl:35-42 -- redefined likewise: like GPU tasks as one batch split over every
#                                                  visible GPU (mcmc_group_*), then stopped (run_serialmc_exit);
#                                                  other arrays pmap as before;
#   ess(cs::Array{MCMCChain})   ess.jl:6-10      -- a new method (the reference's ess(c::MCMCChain) is untouched):
#                                                  the ESS of every chain of a GPU batch in one mcmc_stats_ess call.
# Runner semantics.  A GPU task produces every step (run_serialmc applies the kept range itself), in chunks of at
# most the task runner's len; the samplers' adaptation reads the task's own runner (MALA.jl:116, HMC.jl:167,
# HMCDA.jl:133-141), so the task runner's burnin is set as the chains' tuner burnin (mcmc_chains_set_tuner_burnin)
# apart from the chunks' kept range.  All tasks of one MCMCHipModel share one uploaded model per device.
# Random streams.  The reference's tasks draw from Julia's global RNG as they run, so every spun task samples a
# chain of its own.  A GPU chain's stream is (Philox key, global chain id), so the mirror of the global RNG is
# hip_stream: a key plus a cursor over chain ids (hip_srand(seed) restarts it); a task takes its id when it first
# runs.  Drawn keys carry the top bit (hip_key), explicit seeds of the plain binding (MCMCHip.jl) do not, so the two
# never share a stream.
# Text only in this repository: the image has no Julia.  Struct layouts mirror include/mcmc_hip.h field for field
# (tests/test_api_cpu.py::test_julia_hook_structs_mirror_header checks the field lists against the header).

const hiplib = haskey(ENV, "MCMCHIP_LIB") ? ENV["MCMCHIP_LIB"] : "libmcmc_hip"

export MCMCHipModel, hipmodel, hip_run_batch, hip_run_arrays, hip_srand, hip_ess

# ---- C structs (include/mcmc_hip.h), isbits, C layout
immutable HipModelDesc            # mcmc_model_desc
  kind::Int32; has_gradient::Int32; d::Int64
  init::Ptr{Float64}; scale::Ptr{Float64}
  mu::Float64; sigma::Float64; prior_sigma::Float64; noise_sigma::Float64; link_sign::Float64
  n::Int64; X::Ptr{Float64}; Y::Ptr{Float64}
  dist::Int32
end
immutable HipSamplerCfg           # mcmc_sampler_cfg
  kind::Int32; scale::Float64; drift_step::Float64; n_leaps::Int64; leap_step::Float64
  rate::Float64; len::Float64; shrinkage::Float64; t0::Float64; step::Float64
  tuner::Int32; adapt_step::Int64; max_step::Int64; target_path::Float64; target_rate::Float64
  max_leaps::Int64
end
immutable HipRunnerCfg            # mcmc_runner_cfg
  burnin::Int64; thinning::Int64; len::Int64
end
type HipOutputs                   # mcmc_outputs (the library writes runtime_s, kernel_ms, nkept)
  samples::Ptr{Float64}; gradients::Ptr{Float64}; accept_bits::Ptr{Uint64}
  final_x::Ptr{Float64}; final_lp::Ptr{Float64}; on_device::Int32
  runtime_s::Float64; kernel_ms::Float64; nkept::Int64
end
immutable HipSeqMCCfg             # mcmc_seqmc_cfg
  steps::Int64; burnin::Int64; trigger::Float64
end

const HIP_MODEL_KINDS = {:isonormal_dot => 1, :normal => 2, :logistic => 3, :linear => 4, :absnormal => 5, :dist => 6,
                         :probit => 7, :dist_obs => 8, :ou => 9}
const HIP_DISTS = {:Normal => 1, :Uniform => 2, :Weibull => 3, :Beta => 4, :TDist => 5, :Exponential => 6,
                   :Gamma => 7, :Cauchy => 8, :LogNormal => 9, :Laplace => 10}

hipcheck(st::Cint) = st == 0 ? nothing :
  error(bytestring(ccall((:mcmc_last_error, hiplib), Ptr{Uint8}, ())))   # the reference's @assert texts

# ---- the model: a catalogue entry (Julia closures cannot cross the C ABI) with MCMCLikelihoodModel's metadata
type MCMCHipModel <: MCMCModel
  kind::Symbol
  size::Int                       # model.size
  init::Vector{Float64}           # model.init
  scale::Vector{Float64}          # model.scale
  pmap::Dict                      # model.pmap: column names of the chain's DataFrames (SerialMC.jl:70-80)
  gradient::Bool
  mu::Float64; sigma::Float64     # :normal, :absnormal; :dist parameters p1, p2
  dist::Symbol
  prior_sigma::Float64; noise_sigma::Float64; link_sign::Float64
  X::Matrix{Float64}              # n x d covariates (regressions)
  Y::Vector{Float64}
  device::Int
end

# hipmodel(:isonormal_dot; init=ones(3))                       model(v -> -dot(v,v), grad = v -> -2v, init=...)
# hipmodel(:normal; mu=0., sigma=1., init=zeros(5))             model(:(v ~ Normal(mu, sigma)), v=zeros(5), gradient=true)
# hipmodel(:logistic; X=X, Y=Y, init=zeros(size(X,2)))          examples/logistic_regression.jl:16-22
# hipmodel(:linear; X=X, Y=Y)                                   examples/linear_regression.jl:14-20
# hipmodel(:dist; dist=:Gamma, mu=2., sigma=1., init=ones(3))   model(:(v ~ Gamma(2., 1.)), v=ones(3))
# hipmodel(:probit; X=X, Y=y, prior_sigma=10.)                  examples/probit_regression.jl:18-40
# hipmodel(:dist_obs; dist=:Normal, mu=1., sigma=1., Y=ones(1000), init=[1.])
#                                                               model(:(y = x * v; y ~ Normal(1, 1)), x=1.)
# hipmodel(:ou; Y=x, init=[0.05, 1., 1.], scale=[1000., 1., 10.])
#                                                               examples/ornstein.jl:19-30 (the series x in Y; the
#                                                               chain's columns tau, sigma, mu as model(ex, tau=...) names)
function hipmodel(kind::Symbol; init::Vector{Float64}=Float64[], scale::Vector{Float64}=Float64[],
                  name::Symbol=:vars, gradient::Bool=true, mu::Float64=0., sigma::Float64=1., dist::Symbol=:Normal,
                  prior_sigma::Float64=1., noise_sigma::Float64=1., link_sign::Float64=1.,
                  X::Matrix{Float64}=zeros(0, 0), Y::Vector{Float64}=Float64[], device::Int=0,
                  pmap::Union(Dict, Nothing)=nothing)
  @assert haskey(HIP_MODEL_KINDS, kind) "unknown GPU model kind $kind"
  if kind == :logistic || kind == :linear || kind == :probit
    @assert size(X, 1) == length(Y) "X has $(size(X, 1)) rows, Y $(length(Y)) entries"
    isempty(init) && (init = zeros(size(X, 2)))
  end
  kind == :dist_obs && (@assert length(init) == 1 "y = x * v: x is a scalar"; @assert !isempty(Y) "the data v in Y")
  if kind == :ou
    @assert length(init) == 3 "the Ornstein-Uhlenbeck model has 3 parameters (tau, sigma, mu)"
    @assert length(Y) >= 2 "the Ornstein-Uhlenbeck model needs a series of at least 2 values in Y"
    pmap == nothing && (pmap = {:tau => (1, ()), :sigma => (2, ()), :mu => (3, ())})
  end
  d = length(init)
  @assert d > 0 "init must hold the parameter vector"
  isempty(scale) && (scale = ones(d))
  @assert length(scale) == d "scale parameter size ($(length(scale))) different from initial values ($d)"
  if pmap == nothing
    pmap = d == 1 ? {name => (1, ())} : {name => (1, (d,))}     # one scalar or vector variable, as model() builds
  end
  MCMCHipModel(kind, d, copy(init), copy(scale), pmap, gradient, mu, sigma, dist, prior_sigma, noise_sigma,
               link_sign, X, Y, device)
end

function hip_desc(m::MCMCHipModel, Xr::Vector{Float64})
  HipModelDesc(HIP_MODEL_KINDS[m.kind], m.gradient ? 1 : 0, m.size, pointer(m.init), pointer(m.scale),
               m.mu, m.sigma, m.prior_sigma, m.noise_sigma, m.link_sign, length(m.Y),
               isempty(Xr) ? convert(Ptr{Float64}, C_NULL) : pointer(Xr),
               isempty(m.Y) ? convert(Ptr{Float64}, C_NULL) : pointer(m.Y),
               (m.kind == :dist || m.kind == :dist_obs) ? HIP_DISTS[m.dist] : 0)
end

# ---- samplers (RWM.jl:24-36, MALA.jl:50-62, HMC.jl:53-74, HMCDA.jl:24-43, RAM.jl:22-35)
hip_tuner(t) = t == nothing ? (0, 0, 0, 0., 0.) :
  (1, t.adaptStep, t.maxStep, t.targetPath, t.targetRate)      # EmpiricalMCMCTuner (samplers.jl:32-50)
hip_cfg(kind, scale, drift, nl, ls, rate, len, shr, t0, st, tu, maxl) =
  HipSamplerCfg(kind, scale, drift, nl, ls, rate, len, shr, t0, st, tu[1], tu[2], tu[3], tu[4], tu[5], maxl)
hip_sampler(s::RWM) = (s.tuner == nothing || error("RWM tuners are not built for the GPU");
                       hip_cfg(1, s.scale, 0., 0, 0., 0., 0., 0., 0., 0., hip_tuner(nothing), 0))
hip_sampler(s::MALA) = hip_cfg(2, 0., s.driftStep, 0, 0., 0., 0., 0., 0., 0., hip_tuner(s.tuner), 0)
hip_sampler(s::HMC) = hip_cfg(3, 0., 0., s.nLeaps, s.leapStep, 0., 0., 0., 0., 0., hip_tuner(s.tuner), 0)
hip_sampler(s::HMCDA) = hip_cfg(4, 0., 0., 0, 0., s.rate, s.len, s.shrinkage, s.t0, s.step, hip_tuner(nothing), 0)
hip_sampler(s::RAM) = hip_cfg(5, s.scale, 0., 0, 0., s.rate, 0., 0., 0., 0., hip_tuner(nothing), 0)

# storeLeaps (HMC.jl:145-150, HMCDA.jl:110-117): leapfrog states recorded per step, up to a cap -- the trajectory
# length for HMC (the tuner's maxStep bound when tuned), hip_leap_cap for HMCDA, whose length round(len / leapStep)
# adapts (a longer trajectory is an error rather than a truncated record)
const hip_leap_cap = 1024
hip_store_leaps(s::MCMCSampler) = (isa(s, HMC) || isa(s, HMCDA)) && s.storeLeaps
hip_leaps_cap(s::HMC) = s.tuner == nothing ? s.nLeaps : max(s.nLeaps, s.tuner.maxStep)
hip_leaps_cap(s::HMCDA) = hip_leap_cap

# ---- device objects, released by finalizers (chains before their model, the model before its context: each
#      holds a reference to its parent, so the parent is still reachable while the child is alive)
type HipContext
  h::Ptr{Void}
  function HipContext(dev::Int)
    h = Array(Ptr{Void}, 1)
    hipcheck(ccall((:mcmc_ctx_create, hiplib), Cint, (Cint, Ptr{Ptr{Void}}), dev, h))
    c = new(h[1])
    finalizer(c, x -> (x.h == C_NULL || ccall((:mcmc_ctx_destroy, hiplib), Cint, (Ptr{Void},), x.h); x.h = C_NULL))
    c
  end
end
type HipModelHandle
  h::Ptr{Void}
  ctx::HipContext
  function HipModelHandle(ctx::HipContext, m::MCMCHipModel)
    Xr = isempty(m.X) ? Float64[] : vec(m.X')          # the ABI wants X row-major [n][d] = Julia's X' column-major
    h = Array(Ptr{Void}, 1)
    hipcheck(ccall((:mcmc_model_create, hiplib), Cint, (Ptr{Void}, Ptr{HipModelDesc}, Ptr{Ptr{Void}}),
                   ctx.h, [hip_desc(m, Xr)], h))          # the library copies X, Y, init, scale to the device
    o = new(h[1], ctx)
    finalizer(o, x -> (x.h == C_NULL || ccall((:mcmc_model_destroy, hiplib), Cint, (Ptr{Void},), x.h); x.h = C_NULL))
    o
  end
end
type HipChains
  h::Ptr{Void}
  model::HipModelHandle
  d::Int
  nchains::Int
  function HipChains(mh::HipModelHandle, cfg::HipSamplerCfg, d::Int, nchains::Int, seed::Uint64, offset::Int)
    h = Array(Ptr{Void}, 1)
    hipcheck(ccall((:mcmc_chains_create, hiplib), Cint,
                   (Ptr{Void}, Ptr{HipSamplerCfg}, Int64, Int64, Uint64, Ptr{Float64}, Ptr{Ptr{Void}}),
                   mh.h, [cfg], nchains, offset, seed, convert(Ptr{Float64}, C_NULL), h))   # every chain at init
    hip_chains_owned(new(h[1], mh, d, nchains))
  end
  # chains [first, first + count) of src (0-based first), state and step counter copied: mcmc_chains_fork
  function HipChains(src::HipChains, first::Int, count::Int)
    h = Array(Ptr{Void}, 1)
    hipcheck(ccall((:mcmc_chains_fork, hiplib), Cint, (Ptr{Void}, Int64, Int64, Ptr{Ptr{Void}}),
                   src.h, first, count, h))
    hip_chains_owned(new(h[1], src.model, src.d, count))
  end
end
hip_chains_owned(c::HipChains) =
  (finalizer(c, x -> (x.h == C_NULL || ccall((:mcmc_chains_destroy, hiplib), Cint, (Ptr{Void},), x.h); x.h = C_NULL));
   c)

# MCMC.reset's device side: every chain of ch at x (d x nchains), log-targets returned (mcmc_chains_set_state)
function hip_set_state!(ch::HipChains, x::Matrix{Float64})
  lp = Array(Float64, ch.nchains)
  hipcheck(ccall((:mcmc_chains_set_state, hiplib), Cint, (Ptr{Void}, Ptr{Float64}, Ptr{Float64}),
                 ch.h, x', lp))                  # [d][C] in C order = Julia (C, d)
  lp
end

const hip_contexts = Dict{Int, HipContext}()
hip_context(dev::Int) = haskey(hip_contexts, dev) ? hip_contexts[dev] : (hip_contexts[dev] = HipContext(dev))

# the tuners' burnin of a task's chains: its own runner's (MALA.jl:116, HMC.jl:167, HMCDA.jl:133-141)
hip_set_tuner_burnin!(ch::HipChains, burnin::Int) =
  hipcheck(ccall((:mcmc_chains_set_tuner_burnin, hiplib), Cint, (Ptr{Void}, Int64), ch.h, burnin))
hip_tuner_burnin(r::MCMCRunner) = (isa(r, SerialMC) || isa(r, SeqMC)) ? r.burnin : 0

# one uploaded model (X, Y, init, scale on the device) per MCMCHipModel object, shared by every task spun from it;
# held weakly, so it goes with the model (a task's chains keep their handle alive while they live)
const hip_model_handles = WeakKeyDict()
function hip_model_handle(m::MCMCHipModel)
  if !haskey(hip_model_handles, m) || hip_model_handles[m].ctx.h != hip_context(m.device).h
    hip_model_handles[m] = HipModelHandle(hip_context(m.device), m)
  end
  hip_model_handles[m]
end

hip_chains(m::MCMCHipModel, s::MCMCSampler, nchains::Int, seed::Uint64, offset::Int) =
  HipChains(hip_model_handle(m), hip_sampler(s), m.size, nchains, seed, offset)

# ---- the global stream (see the header): hip_draw(n) takes n consecutive global chain ids; ids are 32-bit (the
#      Philox counter's chain word), so a cursor that would pass 2^32 moves on to the next key.  The Philox key of a
#      drawn stream is hip_key(seed): the top bit set, a key space no explicit seed (< 2^63) reaches
type HipStream
  seed::Int
  next::Int
end
const hip_stream = HipStream(1, 0)
hip_srand(seed::Int) = (hip_stream.seed = seed; hip_stream.next = 0; nothing)
hip_key(seed::Int) = (uint64(seed) & 0x7fffffffffffffff) | 0x8000000000000000
function hip_draw(n::Int)
  if hip_stream.next + n > 2^32
    hip_stream.seed += 1
    hip_stream.next = 0
  end
  first = hip_stream.next
  hip_stream.next += n
  (hip_key(hip_stream.seed), first)
end

# one mcmc_run_serialmc of `len` steps, rows (burnin+1):thinning:len kept: samples / gradients [nkept*d*C]
# ([nkept][d][C] in C order = Julia (C, d, nkept) column-major), accept bits [nkept][ceil(C/64)], the final state
# (C, d) and log-targets; with cap >= 0 the storeLeaps record of every kept step (mcmc_chains_store_leaps):
# pars / grad / m as Julia (C, d, cap+1, nkept), logTarget / H (C, cap+1, nkept), nleaps (C, nkept)
type HipRun
  x::Array{Float64, 3}
  g::Array{Float64, 3}
  bits::Matrix{Uint64}
  fx::Matrix{Float64}
  flp::Vector{Float64}
  runtime::Float64
  leaps::Dict
end
hip_accept(o::HipRun, j::Int, c::Int) = (o.bits[div(c - 1, 64) + 1, j] >> ((c - 1) % 64)) & 1 == 1

function hip_out_arrays(C::Int, d::Int, nk::Int, grads::Bool)
  x = Array(Float64, C, d, nk)
  g = grads ? Array(Float64, C, d, nk) : Array(Float64, 0, 0, 0)
  bits = zeros(Uint64, div(C + 63, 64), nk)
  fx = Array(Float64, C, d)
  flp = Array(Float64, C)
  x, g, bits, fx, flp
end

function hip_run!(ch::HipChains, burnin::Int, thinning::Int, len::Int, grads::Bool, cap::Int=-1)
  nk = length((burnin + 1):thinning:len)
  C, d = ch.nchains, ch.d
  x, g, bits, fx, flp = hip_out_arrays(C, d, nk, grads)
  leaps = Dict()
  if cap >= 0
    for k in (:pars, :grad, :m); leaps[k] = Array(Float64, C, d, cap + 1, nk); end
    for k in (:logTarget, :H); leaps[k] = Array(Float64, C, cap + 1, nk); end
    leaps[:nleaps] = Array(Int32, C, nk)
    hipcheck(ccall((:mcmc_chains_store_leaps, hiplib), Cint,
                   (Ptr{Void}, Int64, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                   ch.h, cap, leaps[:pars], leaps[:grad], leaps[:m], leaps[:logTarget], leaps[:H], leaps[:nleaps]))
  end
  out = HipOutputs(pointer(x), grads ? pointer(g) : convert(Ptr{Float64}, C_NULL), pointer(bits),
                   pointer(fx), pointer(flp), 0, 0., 0., 0)
  hipcheck(ccall((:mcmc_run_serialmc, hiplib), Cint, (Ptr{Void}, Ptr{HipRunnerCfg}, Ptr{HipOutputs}),
                 ch.h, [HipRunnerCfg(burnin, thinning, len)], &out))
  HipRun(x, g, bits, fx, flp, out.runtime_s, leaps)
end

# ---- one node's GPUs (mcmc_group_*, the prun replacement, runners.jl:35-42): one batch of n chains split into
#      contiguous 64-chain-aligned blocks, one per device, every block's step loop concurrently, each block's outputs
#      copied device -> host into its columns of the arrays; bit-identical to one context running every chain
type HipGroup
  h::Ptr{Void}
  function HipGroup(devs::Vector{Int32})
    h = Array(Ptr{Void}, 1)
    hipcheck(ccall((:mcmc_group_create, hiplib), Cint, (Ptr{Int32}, Int32, Ptr{Ptr{Void}}), devs, length(devs), h))
    g = new(h[1])
    finalizer(g, x -> (x.h == C_NULL || ccall((:mcmc_group_destroy, hiplib), Cint, (Ptr{Void},), x.h); x.h = C_NULL))
    g
  end
end
function hip_devices()
  n = Array(Cint, 1)
  hipcheck(ccall((:mcmc_device_count, hiplib), Cint, (Ptr{Cint},), n))
  Int32[0:(n[1] - 1)]
end
const hip_groups = Dict{Vector{Int32}, HipGroup}()
hip_group(devs::Vector{Int32}) = haskey(hip_groups, devs) ? hip_groups[devs] : (hip_groups[devs] = HipGroup(devs))

function hip_run_group(m::MCMCHipModel, s::MCMCSampler, r::SerialMC, n::Int, seed::Uint64, first::Int,
                       devs::Vector{Int32})
  g = hip_group(devs)
  Xr = isempty(m.X) ? Float64[] : vec(m.X')
  desc = [hip_desc(m, Xr)]                                # model uploaded once per device by the library
  h = Array(Ptr{Void}, 1)
  hipcheck(ccall((:mcmc_group_chains_create, hiplib), Cint,
                 (Ptr{Void}, Ptr{HipModelDesc}, Ptr{HipSamplerCfg}, Int64, Int64, Uint64, Ptr{Float64}, Ptr{Ptr{Void}}),
                 g.h, desc, [hip_sampler(s)], n, first, seed, convert(Ptr{Float64}, C_NULL), h))
  length(Xr) + length(m.Y) + length(m.init) + length(m.scale)   # the descriptor's arrays stay rooted to here
  try
    x, gr, bits, fx, flp = hip_out_arrays(n, m.size, length(r.r), has_grads(s))
    out = HipOutputs(pointer(x), has_grads(s) ? pointer(gr) : convert(Ptr{Float64}, C_NULL), pointer(bits),
                     pointer(fx), pointer(flp), 0, 0., 0., 0)
    gather = Array(Float64, 1)
    hipcheck(ccall((:mcmc_group_run_serialmc, hiplib), Cint,
                   (Ptr{Void}, Ptr{HipRunnerCfg}, Ptr{HipOutputs}, Ptr{Float64}),
                   h[1], [HipRunnerCfg(r.burnin, r.thinning, r.len)], &out, gather))
    HipRun(x, gr, bits, fx, flp, out.runtime_s, Dict())
  finally
    ccall((:mcmc_group_chains_destroy, hiplib), Cint, (Ptr{Void},), h[1])   # prun's tasks come back stopped
  end
end

has_grads(s::MCMCSampler) = isa(s, MALA) || isa(s, HMC) || isa(s, HMCDA)

# diagnostics["leaps"] of kept step j, chain c: the reference's leapStates, HMCSample(pars, grad, m, logTarget, H)
# for leap 0 (state0 after update!) .. nLeaps
function hip_leap_states(o::HipRun, j::Int, c::Int, cap::Int)
  nl = int(o.leaps[:nleaps][c, j])
  nl > cap && error("storeLeaps: a trajectory of $nl leapfrogs exceeds the recording cap $cap")
  L = o.leaps
  HMCSample[HMCSample(vec(L[:pars][c, :, l, j]), vec(L[:grad][c, :, l, j]), vec(L[:m][c, :, l, j]),
                      L[:logTarget][c, l, j], L[:H][c, l, j]) for l in 1:(nl + 1)]
end

# ---- per-task state, shared by a GPU task's producer loop and the batched runners (hip_tasks maps the Julia Task
#      of an MCMCTask to it)
type HipTaskState
  model::MCMCHipModel
  sampler::MCMCSampler
  runner::MCMCRunner                  # the task's runner: its burnin drives the tuners, its len the chunk length
  chains::Union(HipChains, Nothing)   # the task's one GPU chain, made on first use
  src::Union(HipChains, Nothing)      # after a batched run: the batch, whose chain `first` this task continues
  first::Int
  seed::Uint64
  offset::Int                         # global chain id; -1 until drawn
  stopped::Bool
  buf::Union(HipRun, Nothing)         # chunk mode: steps run ahead on the GPU, produced one by one
  pos::Int
  single::Bool                        # after a reset: one GPU step per consume, with the log-targets it produced
  x::Vector{Float64}
  lp::Float64
end
HipTaskState(m::MCMCHipModel, s::MCMCSampler, r::MCMCRunner) =
  HipTaskState(m, s, r, nothing, nothing, 0, uint64(0), -1, false, nothing, 0, false, Float64[], NaN)
const hip_tasks = WeakKeyDict()

function hip_ensure!(st::HipTaskState)
  st.stopped && error("the task was stopped by prun (run_serialmc_exit, SerialMC.jl:87-91)")
  st.chains != nothing && return st.chains
  if st.src != nothing                                   # continue chain `first` of a batched run
    st.chains = HipChains(st.src, st.first, 1)
    st.src = nothing
  else
    st.seed, st.offset = hip_draw(1)
    st.chains = hip_chains(st.model, st.sampler, 1, st.seed, st.offset)
  end
  # every step is kept by the chunk runs (hip_produce_loop), so the adaptation window is set apart: the task
  # runner's burnin (MALA.jl:116, HMC.jl:167, HMCDA.jl:133-141)
  hip_set_tuner_burnin!(st.chains, hip_tuner_burnin(st.runner))
  st.chains
end

# the :reset hook: the chain jumps to x, its log-target re-evaluated there (the samplers' hooks, RWM.jl:49,
# MALA.jl:75-80, HMC.jl:114-116, HMCDA.jl:82-83, RAM.jl:47); buffered steps are dropped and the task turns to one
# GPU step per consume, so that every MCMCSample carries plogtarget and logtarget (SeqMC.jl:69-72 reads them)
function hip_reset!(st::HipTaskState, x::Vector{Float64})
  ch = hip_ensure!(st)
  st.lp = hip_set_state!(ch, reshape(copy(x), length(x), 1))[1]
  st.x = copy(x)
  st.buf = nothing
  st.single = true
  nothing
end

# ---- drop-in: spinTask for GPU models.  The Julia Task produces one MCMCSample per step, as SamplerTask does:
#      from GPU runs of `chunk` steps (every step kept; plogtarget / pars / logtarget NaN: run_serialmc reads only
#      ppars, pgrads and diagnostics), or, after MCMC.reset, from single GPU steps with their log-targets.
#      A continuation (run(c), runners.jl:14) keeps consuming the same task, i.e. the same GPU chain.
#      A chunk is at most the task runner's len (one run(t) consumes exactly len steps: nothing runs ahead of what
#      run_serialmc takes), capped at hip_chunk; a task whose runner is not SerialMC (consumed one sample at a time
#      by run_seqmc / run_serialtempmc) steps one at a time.
const hip_chunk = 1000
function hip_chunk_len(st::HipTaskState, cap::Int)
  n = isa(st.runner, SerialMC) ? min(hip_chunk, st.runner.len) : 1
  cap < 0 ? n : max(1, min(n, div(1 << 28, 8 * (cap + 1) * (3 * st.model.size + 2))))
end

function hip_produce_loop(st::HipTaskState)
  task_local_storage(:reset, (resetPars::Vector{Float64}) -> hip_reset!(st, resetPars))
  grads = has_grads(st.sampler)
  cap = hip_store_leaps(st.sampler) ? hip_leaps_cap(st.sampler) : -1
  nan = fill(NaN, st.model.size)
  while true
    ch = hip_ensure!(st)
    if st.single
      o = hip_run!(ch, 0, 1, 1, grads, cap)
      diag = Dict{Any, Any}()
      diag["accept"] = hip_accept(o, 1, 1)
      cap >= 0 && (diag["leaps"] = hip_leap_states(o, 1, 1, cap))
      x1, lp1 = vec(o.fx[1, :]), o.flp[1]
      produce(MCMCSample(x1, lp1, grads ? vec(o.g[1, :, 1]) : nothing, st.x, st.lp, nothing, diag))
      st.x, st.lp = x1, lp1
    else
      if st.buf == nothing || st.pos > size(st.buf.x, 3)
        st.buf = hip_run!(ch, 0, 1, hip_chunk_len(st, cap), grads, cap)
        st.pos = 1
      end
      o, j = st.buf, st.pos
      st.pos += 1
      diag = Dict{Any, Any}()
      diag["accept"] = hip_accept(o, j, 1)
      cap >= 0 && (diag["leaps"] = hip_leap_states(o, j, 1, cap))
      produce(MCMCSample(vec(o.x[1, :, j]), NaN, grads ? vec(o.g[1, :, j]) : nothing, nan, NaN, nothing, diag))
    end
  end
end

function spinTask(m::MCMCHipModel, s::MCMCSampler, r::MCMCRunner)
  hip_sampler(s)                                         # refuse unsupported configurations now, as the ctor would
  st = HipTaskState(m, s, r)
  task = Task(() -> hip_produce_loop(st))
  hip_tasks[task] = st
  MCMCTask(task, m, s, r)
end

# ---- batched: like tasks as one chain batch
function hip_colnames(m::MCMCHipModel)
  cn = Array(ASCIIString, m.size)
  for (k, v) in m.pmap
    if length(v[2]) == 0
      cn[v[1]] = string(k)
    elseif length(v[2]) == 1
      for i in 1:v[2][1]; cn[v[1] + i - 1] = "$k.$i"; end
    else
      for j in 1:v[2][2], i in 1:v[2][1]; cn[v[1] + (j - 1) * v[2][1] + i - 1] = "$k.$i.$j"; end
    end
  end
  cn
end

# chain c of a batched run, built like run_serialmc's (SerialMC.jl:37-85): samples / gradients DataFrames with the
# pmap column names, diagnostics {"step" => collect(r), "accept" => Bool[] (, "leaps")}, the batch's runTime
function hip_chain(m::MCMCHipModel, s::MCMCSampler, r::SerialMC, o::HipRun, c::Int, t::MCMCTask)
  cn = hip_colnames(m)
  nk = size(o.x, 3)
  sc = reshape(o.x[c, :, :], m.size, nk)'                               # nkept x d
  gd = has_grads(s) ? DataFrame(reshape(o.g[c, :, :], m.size, nk)', cn) : DataFrame()
  diags = {"step" => collect(r.r), "accept" => Bool[hip_accept(o, j, c) for j in 1:nk]}
  if hip_store_leaps(s)
    cap = hip_leaps_cap(s)
    diags["leaps"] = Array{HMCSample}[hip_leap_states(o, j, c, cap) for j in 1:nk]
  end
  MCMCChain(r.r, DataFrame(sc, cn), gd, diags, t, o.runtime)
end

# tasks that can share one batch: GPU tasks of one model object, one sampler configuration and one SerialMC runner,
# none started yet
function hip_batchable(t::Array{MCMCTask})
  isempty(t) && return false
  t1 = t[1]
  isa(t1.model, MCMCHipModel) && isa(t1.runner, SerialMC) || return false
  cfg1 = hip_sampler(t1.sampler)
  for x in t
    haskey(hip_tasks, x.task) || return false
    st = hip_tasks[x.task]
    (st.chains == nothing && st.src == nothing && !st.stopped) || return false
    (x.model === t1.model && isa(x.runner, SerialMC)) || return false
    (x.runner.burnin, x.runner.thinning, x.runner.len) == (t1.runner.burnin, t1.runner.thinning, t1.runner.len) ||
      return false
    (hip_sampler(x.sampler) == cfg1 && hip_store_leaps(x.sampler) == hip_store_leaps(t1.sampler)) || return false
  end
  true
end

# one mcmc_run_serialmc for every task of t (consecutive global chain ids from the stream); task k then continues
# chain k (a fork of the batch's state on its first use) or, with stop (prun), is stopped (run_serialmc_exit)
#      (prun: over the devices `devs` as one mcmc_group when there are several; storeLeaps records stay on one device)
function hip_run_tasks(t::Array{MCMCTask}, stop::Bool, devs::Vector{Int32}=Int32[])
  m, s, r = t[1].model, t[1].sampler, t[1].runner
  n = length(t)
  seed, first = hip_draw(n)
  ch = nothing
  if stop && length(devs) > 1 && !hip_store_leaps(s)
    o = hip_run_group(m, s, r, n, seed, first, devs)
  else
    ch = hip_chains(m, s, n, seed, first)
    cap = hip_store_leaps(s) ? hip_leaps_cap(s) : -1
    o = hip_run!(ch, r.burnin, r.thinning, r.len, has_grads(s), cap)
  end
  res = Array(MCMCChain, size(t))
  for k in 1:n
    st = hip_tasks[t[k].task]
    st.seed, st.offset = seed, first + k - 1
    if stop
      st.stopped = true
    else
      st.src, st.first = ch, k - 1
    end
    res[k] = hip_chain(m, s, r, o, k, t[k])
    stop && stop!(res[k])
  end
  res
end

# run(t::Array{MCMCTask}) (runners.jl:17-33): like GPU tasks as one batch; every other array as the reference runs it
function run(t::Array{MCMCTask}; args...)
  lastrunner = t[end].runner
  @assert all(map(x -> isa(x.runner, typeof(lastrunner)), t)) "Runners do not have the same runner type"
  isa(lastrunner, SerialMC) && hip_batchable(t) && return hip_run_tasks(t, false)
  isa(lastrunner, SeqMC) && hip_seqmc_able(t) && return hip_run_seqmc(t; args...)
  if isa(lastrunner, SerialMC)
    res = Array(MCMCChain, size(t))
    for i in 1:length(t); res[i] = run(t[i]); end
    return res
  end
  isa(lastrunner, SerialTempMC) && return run_serialtempmc(t)
  run_seqmc(t; args...)
end

# prun(t::Array{MCMCTask}) (runners.jl:35-42): like GPU tasks as one batch, then stopped; others pmap as before
function prun(t::Array{MCMCTask}; args...)
  lastrunner = t[end].runner
  @assert all(map(x -> isa(x.runner, typeof(lastrunner)), t)) "Runners do not have the same runner type"
  isa(lastrunner, SerialMC) || return nothing
  hip_batchable(t) && return hip_run_tasks(t, true, hip_devices())
  pmap(run_serialmc_exit, t)
end

# ---- SeqMC (SeqMC.jl:39-122) on the GPU: GPU targets, none started, one parameter size
function hip_seqmc_able(t::Array{MCMCTask})
  isempty(t) && return false
  for x in t
    (isa(x.model, MCMCHipModel) && haskey(hip_tasks, x.task)) || return false
    st = hip_tasks[x.task]
    (st.chains == nothing && st.src == nothing && !st.stopped) || return false
  end
  true
end

# Philox key of target k's chains (mcmchip.seqmc.target_seed on the drawn key, kept in the drawn key space)
hip_target_key(seed::Uint64, k::Int) = ((seed + uint64(k + 1) * 0x9e3779b97f4a7c15) & 0x7fffffffffffffff) |
                                       0x8000000000000000

# run_seqmc(targets; particles) as one mcmc_run_seqmc: particle n is chain n of every target's chain batch; per outer
# step and target every particle is reset into the target (MCMC.reset) and advanced one step of its sampler, the
# weights updated and, when var(W) < trigger, the particles resampled -- on the device, no host round trip inside the
# loop.  The chain is the reference's: samples (steps - burnin) * npart rows, step-major; diagnostics "weigths" (sic,
# SeqMC.jl:119) and "particle"; its range the reference's own (burnin+1):1:((steps-burnin)*npart) (SeqMC.jl:116).
# The particles' chains and the resampling draws come from the global stream (hip_draw): a fresh population stream.
function hip_run_seqmc(targets::Array{MCMCTask}; particles::Vector{Vector{Float64}} = [[randn()] for i in 1:100])
  ntargets = length(targets)
  npart = length(particles)
  tsize = targets[end].model.size
  r = targets[end].runner
  @assert all(map(t -> t.model.size, targets) .== tsize) "Models do not have the same parameter vector size"
  @assert all(map(p -> length(p), particles) .== tsize) "particles must have $tsize coordinates"
  seed, first = hip_draw(npart)
  chs = HipChains[HipChains(hip_model_handle(targets[k].model), hip_sampler(targets[k].sampler), tsize, npart,
                            hip_target_key(seed, k - 1), first) for k in 1:ntargets]
  P = Float64[particles[n][j] for n in 1:npart, j in 1:tsize]           # [d][npart] in C order
  nst = r.steps - r.burnin
  S = Array(Float64, npart, tsize, nst)                                  # [nst][d][npart]
  W = Array(Float64, npart, nst)                                         # [nst][npart]
  F = zeros(Int32, ntargets, r.steps)                                    # resampled flags [steps][ntargets]
  rt = Array(Float64, 1)
  hipcheck(ccall((:mcmc_run_seqmc, hiplib), Cint,
                 (Ptr{Ptr{Void}}, Int32, Int64, Ptr{Float64}, Ptr{HipSeqMCCfg}, Uint64, Int32, Ptr{Float64},
                  Ptr{Float64}, Ptr{Int32}, Ptr{Float64}),
                 Ptr{Void}[c.h for c in chs], ntargets, npart, P, [HipSeqMCCfg(r.steps, r.burnin, r.trigger)], seed,
                 0, S, W, F, rt))
  M = Array(Float64, nst * npart, tsize)
  for i in 1:nst, j in 1:tsize, n in 1:npart
    M[(i - 1) * npart + n, j] = S[n, j, i]
  end
  MCMCChain((r.burnin + 1):1:((r.steps - r.burnin) * npart), DataFrame(M, hip_colnames(targets[end].model)),
            DataFrame(), {"weigths" => vec(W), "particle" => rep([1:npart], nst), "resampled" => F'}, targets, rt[1])
end

# ---- ESS on the device (ess.jl:6-10 with var.jl's IMSE / IPSE / batch means; mcmc_stats_ess)
const HIP_VTYPES = {:imse => 1, :ipse => 2, :bm => 3}

# samples as hip_run_arrays returns them, (C, d, nkept): ESS and the vtype variance of the mean, each (C, d)
function hip_ess(x::Array{Float64, 3}; vtype::Symbol=:imse, maxlag::Int=0, batchlen::Int=100, device::Int=0)
  @assert haskey(HIP_VTYPES, vtype) "Unknown ESS type $vtype"
  C, d, nk = size(x)
  e, v = Array(Float64, C, d), Array(Float64, C, d)
  hipcheck(ccall((:mcmc_stats_ess, hiplib), Cint,
                 (Ptr{Void}, Ptr{Float64}, Int64, Int64, Int64, Int32, Int64, Int64, Int32, Ptr{Float64}, Ptr{Float64}),
                 hip_context(device).h, x, nk, d, C, HIP_VTYPES[vtype], maxlag, batchlen, 0, e, v))
  e, v
end

# ess(c) of every chain of an array; chains of GPU tasks with equal shapes go to the device in one call, as ess(c)
# would give each (ess.jl:6-10: nrow * var_iid / var_vtype over every column); anything else chain by chain
function ess(cs::Array{MCMCChain}; vtype::Symbol=:imse, maxlag::Int=0, batchlen::Int=100)
  gpu = !isempty(cs) && all(c -> isa(c.task, MCMCTask) && isa(c.task.model, MCMCHipModel), cs)
  if gpu
    nk, d = size(cs[1].samples)
    gpu = all(c -> size(c.samples) == (nk, d), cs)
  end
  if !gpu
    return [vtype == :bm ? ess(c; vtype=vtype, batchlen=batchlen) :
            maxlag > 0 ? ess(c; vtype=vtype, maxlag=maxlag) : ess(c; vtype=vtype) for c in cs]
  end
  x = Float64[cs[c].samples[k, j] for c in 1:length(cs), j in 1:d, k in 1:nk]
  e, _ = hip_ess(x; vtype=vtype, maxlag=maxlag, batchlen=batchlen, device=cs[1].task.model.device)
  [vec(e[c, :]) for c in 1:length(cs)]
end

# nchains independent chains as one batch, each returned MCMCChain's task continuing its own chain
hip_run_batch(m::MCMCHipModel, s::MCMCSampler, r::SerialMC, nchains::Int) =
  run(MCMCTask[spinTask(m, s, r) for i in 1:nchains])

# raw arrays: samples / gradients (C, d, nkept), accept (nkept, C) Bool, runTime -- for batches whose per-chain
# DataFrames would not fit in host memory; the chains come from the global stream
function hip_run_arrays(m::MCMCHipModel, s::MCMCSampler, r::SerialMC, nchains::Int)
  seed, first = hip_draw(nchains)
  devs = hip_devices()
  o = (length(devs) > 1 && nchains >= 64 * length(devs)) ? hip_run_group(m, s, r, nchains, seed, first, devs) :
      hip_run!(hip_chains(m, s, nchains, seed, first), r.burnin, r.thinning, r.len, has_grads(s))
  nk = size(o.x, 3)
  o.x, o.g, Bool[hip_accept(o, j, c) for j in 1:nk, c in 1:nchains], o.runtime
end
