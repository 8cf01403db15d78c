# mcmc_jl_hook.jl -- the MCMC.jl-side dispatch hook: `run(m * s * SerialMC(...))` on the GPU.
#
# Target: the Julia the reference package is written for (Julia 0.3 syntax: `immutable`/`type`, `Union(...)`,
# `{...}` Any-dicts, `Ptr{Void}`, `Uint8`, `finalizer(x, f)`, tasks with produce/consume).  It is include()d into
# module MCMC, after src/runners/SerialMC.jl (INTEGRATION.md §Julia hook shows the one line), so it sees MCMCModel,
# MCMCTask, MCMCChain, MCMCSample, SerialMC, RWM, MALA, HMC, HMCDA, RAM and EmpiricalMCMCTuner directly.  For
# Julia >= 1.0 hosts without MCMC.jl, MCMCHip.jl is the plain binding of the same C ABI.
#
# What it replaces, with no edit to the reference's own files:
#   spinTask(m, s, r)         samplers.jl:53  -- a method for MCMCHipModel (more specific than MCMCModel): the task
#                                                it returns produces MCMCSamples from GPU chains instead of
#                                                SamplerTask's CPU loop, so `m * s * r` (MCMC.jl:87-98), run(t)
#                                                and run_serialmc (runners.jl:7-11, SerialMC.jl:37-85), run(c) (the
#                                                continuation, runners.jl:14) and resume (SerialMC.jl:93-97) all
#                                                run unchanged on top of it;
#   run(t::Array{MCMCTask})   runners.jl:17-33 -- hip_run_batch(m, s, r, nchains) instead: ONE batched launch of
#                                                nchains independent chains (the reference's array of tasks, one
#                                                chain each), returned as an Array{MCMCChain} built like
#                                                run_serialmc's (DataFrame samples / gradients named from pmap,
#                                                diagnostics {"step", "accept"}, runTime), or as raw arrays
#                                                (hip_run_arrays) when a million DataFrames would not fit.
# Text only in this repository: the image has no Julia.  Struct layouts mirror include/mcmc_hip.h field for field
# (tests/test_api_cpu.py::test_julia_hook_structs_mirror_header checks the field lists against the header).

const hiplib = haskey(ENV, "MCMCHIP_LIB") ? ENV["MCMCHIP_LIB"] : "libmcmc_hip"

export MCMCHipModel, hipmodel, hip_run_batch, hip_run_arrays

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

const HIP_MODEL_KINDS = {:isonormal_dot => 1, :normal => 2, :logistic => 3, :linear => 4, :absnormal => 5, :dist => 6,
                         :probit => 7, :dist_obs => 8}
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
function hipmodel(kind::Symbol; init::Vector{Float64}=Float64[], scale::Vector{Float64}=Float64[],
                  name::Symbol=:vars, gradient::Bool=true, mu::Float64=0., sigma::Float64=1., dist::Symbol=:Normal,
                  prior_sigma::Float64=1., noise_sigma::Float64=1., link_sign::Float64=1.,
                  X::Matrix{Float64}=zeros(0, 0), Y::Vector{Float64}=Float64[], device::Int=0)
  @assert haskey(HIP_MODEL_KINDS, kind) "unknown GPU model kind $kind"
  if kind == :logistic || kind == :linear || kind == :probit
    @assert size(X, 1) == length(Y) "X has $(size(X, 1)) rows, Y $(length(Y)) entries"
    isempty(init) && (init = zeros(size(X, 2)))
  end
  kind == :dist_obs && (@assert length(init) == 1 "y = x * v: x is a scalar"; @assert !isempty(Y) "the data v in Y")
  d = length(init)
  @assert d > 0 "init must hold the parameter vector"
  isempty(scale) && (scale = ones(d))
  @assert length(scale) == d "scale parameter size ($(length(scale))) different from initial values ($d)"
  pmap = d == 1 ? {name => (1, ())} : {name => (1, (d,))}       # one scalar or vector variable, as model() builds
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
hip_cfg(kind, scale, drift, nl, ls, rate, len, shr, t0, st, tu) =
  HipSamplerCfg(kind, scale, drift, nl, ls, rate, len, shr, t0, st, tu[1], tu[2], tu[3], tu[4], tu[5], 0)
hip_sampler(s::RWM) = (s.tuner == nothing || error("RWM tuners are not built for the GPU");
                       hip_cfg(1, s.scale, 0., 0, 0., 0., 0., 0., 0., 0., hip_tuner(nothing)))
hip_sampler(s::MALA) = hip_cfg(2, 0., s.driftStep, 0, 0., 0., 0., 0., 0., 0., hip_tuner(s.tuner))
# storeLeaps (HMC.jl:145-150): the C ABI records trajectories (mcmc_chains_store_leaps); this hook does not map them
# into diagnostics["leaps"] yet, so it refuses rather than drop them
hip_sampler(s::HMC) = (s.storeLeaps && error("storeLeaps: use MCMCHip.jl / mcmc_chains_store_leaps");
                       hip_cfg(3, 0., 0., s.nLeaps, s.leapStep, 0., 0., 0., 0., 0., hip_tuner(s.tuner)))
hip_sampler(s::HMCDA) = (s.storeLeaps && error("storeLeaps: use MCMCHip.jl / mcmc_chains_store_leaps");
                         hip_cfg(4, 0., 0., 0, 0., s.rate, s.len, s.shrinkage, s.t0, s.step, hip_tuner(nothing)))
hip_sampler(s::RAM) = hip_cfg(5, s.scale, 0., 0, 0., s.rate, 0., 0., 0., 0., hip_tuner(nothing))

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
  function HipChains(mh::HipModelHandle, cfg::HipSamplerCfg, d::Int, nchains::Int, seed::Int, offset::Int)
    h = Array(Ptr{Void}, 1)
    hipcheck(ccall((:mcmc_chains_create, hiplib), Cint,
                   (Ptr{Void}, Ptr{HipSamplerCfg}, Int64, Int64, Uint64, Ptr{Float64}, Ptr{Ptr{Void}}),
                   mh.h, [cfg], nchains, offset, seed, convert(Ptr{Float64}, C_NULL), h))   # every chain at init
    c = new(h[1], mh, d, nchains)
    finalizer(c, x -> (x.h == C_NULL || ccall((:mcmc_chains_destroy, hiplib), Cint, (Ptr{Void},), x.h); x.h = C_NULL))
    c
  end
end

const hip_contexts = Dict{Int, HipContext}()
hip_context(dev::Int) = haskey(hip_contexts, dev) ? hip_contexts[dev] : (hip_contexts[dev] = HipContext(dev))

hip_chains(m::MCMCHipModel, s::MCMCSampler, nchains::Int, seed::Int) =
  HipChains(HipModelHandle(hip_context(m.device), m), hip_sampler(s), m.size, nchains, seed, 0)

# one mcmc_run_serialmc of `len` steps, rows (burnin+1):thinning:len kept: samples / gradients [nkept*d*C]
# ([nkept][d][C] in C order = Julia (C, d, nkept) column-major), accept bits [nkept][ceil(C/64)]
function hip_run!(ch::HipChains, burnin::Int, thinning::Int, len::Int, grads::Bool)
  nk = length((burnin + 1):thinning:len)
  C, d, nw = ch.nchains, ch.d, div(ch.nchains + 63, 64)
  x = Array(Float64, C, d, nk)
  g = grads ? Array(Float64, C, d, nk) : Array(Float64, 0, 0, 0)
  bits = Array(Uint64, nw, nk)
  out = HipOutputs(pointer(x), grads ? pointer(g) : convert(Ptr{Float64}, C_NULL), pointer(bits),
                   convert(Ptr{Float64}, C_NULL), convert(Ptr{Float64}, C_NULL), 0, 0., 0., 0)
  hipcheck(ccall((:mcmc_run_serialmc, hiplib), Cint, (Ptr{Void}, Ptr{HipRunnerCfg}, Ptr{HipOutputs}),
                 ch.h, [HipRunnerCfg(burnin, thinning, len)], &out))
  accept(j, c) = (bits[div(c - 1, 64) + 1, j] >> ((c - 1) % 64)) & 1 == 1
  x, g, accept, out.runtime_s
end

has_grads(s::MCMCSampler) = isa(s, MALA) || isa(s, HMC) || isa(s, HMCDA)

# ---- drop-in: spinTask for GPU models.  The Julia Task produces one MCMCSample per step, as SamplerTask does,
#      from GPU runs of `chunk` steps (every step kept); run_serialmc consumes them and builds the MCMCChain
#      itself.  plogtarget / pars / logtarget carry NaN: run_serialmc reads only ppars, pgrads and diagnostics.
#      A continuation (run(c), runners.jl:14) keeps consuming the same task, i.e. the same GPU chain.
const hip_chunk = 1000
function spinTask(m::MCMCHipModel, s::MCMCSampler, r::MCMCRunner)
  seed = 1
  task = Task(() -> begin
    ch = hip_chains(m, s, 1, seed)
    grads = has_grads(s)
    nan = fill(NaN, m.size)
    while true
      x, g, accept, _ = hip_run!(ch, 0, 1, hip_chunk, grads)
      for j in 1:hip_chunk
        diag = Dict{Any, Any}()
        diag["accept"] = accept(j, 1)
        produce(MCMCSample(vec(x[1, :, j]), NaN, grads ? vec(g[1, :, j]) : nothing, nan, NaN, nothing, diag))
      end
    end
  end)
  MCMCTask(task, m, s, r)
end

# ---- batched: nchains independent chains in one launch (the reference: an Array{MCMCTask}, one chain each)
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

# raw arrays: samples / gradients (C, d, nkept), accept (nkept, C) Bool, runTime -- for batches whose per-chain
# DataFrames would not fit in host memory
function hip_run_arrays(m::MCMCHipModel, s::MCMCSampler, r::SerialMC, nchains::Int; seed::Int=1)
  ch = hip_chains(m, s, nchains, seed)
  x, g, accept, rt = hip_run!(ch, r.burnin, r.thinning, r.len, has_grads(s))
  nk = size(x, 3)
  acc = Bool[accept(j, c) for j in 1:nk, c in 1:nchains]
  x, g, acc, rt
end

# an Array{MCMCChain}, chain c built like run_serialmc's (SerialMC.jl:37-85): samples / gradients DataFrames with
# the pmap column names, diagnostics {"step" => collect(r), "accept" => Bool[]}, the batch's runTime; each chain's
# task field is a spinTask of its own (a continuation of it restarts a single GPU chain from model.init)
function hip_run_batch(m::MCMCHipModel, s::MCMCSampler, r::SerialMC, nchains::Int; seed::Int=1)
  x, g, acc, rt = hip_run_arrays(m, s, r, nchains; seed=seed)
  cn = hip_colnames(m)
  grads = has_grads(s)
  res = Array(MCMCChain, nchains)
  for c in 1:nchains
    sc = x[c, :, :]; sc = reshape(sc, size(sc, 2), size(sc, 3))'          # nkept x d
    diags = {"step" => collect(r.r), "accept" => acc[:, c]}
    gd = grads ? (gc = reshape(g[c, :, :], m.size, size(g, 3))'; DataFrame(gc, cn)) : DataFrame()
    res[c] = MCMCChain(r.r, DataFrame(sc, cn), gd, diags, spinTask(m, s, r), rt)
  end
  res
end
