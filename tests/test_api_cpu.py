"""CPU tests of the host API and the C ABI boundary (no compute calls: there is no GPU here).

Covers the reference's constructor @asserts (RWM.jl:29, MALA.jl:55, HMC.jl:60-61,
HMCDA.jl:33-36, samplers.jl:40-42, SerialMC.jl:25-27), the MALA-without-gradient
error (test/test_syntax.jl:75, README.md:224), the `*` composition (MCMC.jl:87-98),
DSL parameter packing (test/dsl/unit_tests.jl:29-34), and that libmcmc_hip.so loads
and exports every symbol include/mcmc_hip.h declares.
"""
import ctypes as ct
import os
import re

import numpy as np
import pytest

import mcmchip as mc
from mcmchip import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mcmc_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int)\s+(mcmc_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_lib.EXPORTED_SYMBOLS) == syms
    assert lib.mcmc_abi_version() == 1


def test_model_kinds_agree_across_header_python_and_julia():
    """MCMC_MODEL_* of include/mcmc_hip.h == mcmchip._lib.MODEL_* == MCMCHip.jl's MODEL_* constants."""
    src = open(os.path.join(ROOT, "include", "mcmc_hip.h")).read()
    hdr = {k: int(v) for k, v in re.findall(r"MCMC_MODEL_(\w+)\s*=\s*(\d+)", src)}
    assert len(hdr) == 9 and hdr["OU"] == 9
    jl = open(os.path.join(ROOT, "mcmc.jl_amd", "julia", "MCMCHip.jl")).read()
    jlc = {}
    for names, vals in re.findall(r"^const ((?:MODEL_\w+,?\s*)+)=\s*([\d,\s]+)$", jl, flags=re.M):
        for n, v in zip([x.strip() for x in names.split(",") if x.strip()], vals.split(",")):
            jlc[n[len("MODEL_"):]] = int(v)
    for k, v in hdr.items():
        assert getattr(_lib, "MODEL_" + k) == v, k
        assert jlc[k] == v, k


def test_struct_layouts_match_header():
    # sizes of the C structs (LP64): checked against a compiled probe of the header
    assert ct.sizeof(_lib.RunnerCfg) == 24
    assert ct.sizeof(_lib.ModelDesc) == 4 + 4 + 8 + 8 + 8 + 5 * 8 + 8 + 8 + 8 + 8   # dist: int32 + pad
    assert ct.sizeof(_lib.SamplerCfg) == 4 + 4 + 8 + 8 + 8 + 8 + 5 * 8 + 4 + 4 + 8 + 8 + 8 + 8 + 8
    assert ct.sizeof(_lib.Outputs) == 5 * 8 + 8 + 8 + 8 + 8


def test_header_struct_sizes_compiled(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text('#include "mcmc_hip.h"\n#include <stdio.h>\nint main(void){printf("%zu %zu %zu %zu\\n",'
                   'sizeof(mcmc_model_desc),sizeof(mcmc_sampler_cfg),sizeof(mcmc_runner_cfg),sizeof(mcmc_outputs));'
                   'return 0;}\n')
    exe = tmp_path / "probe"
    assert os.system(f"gcc -I{ROOT}/include {src} -o {exe}") == 0
    out = os.popen(str(exe)).read().split()
    assert [int(v) for v in out] == [ct.sizeof(_lib.ModelDesc), ct.sizeof(_lib.SamplerCfg),
                                     ct.sizeof(_lib.RunnerCfg), ct.sizeof(_lib.Outputs)]


def test_validation_mirrors_reference_asserts():
    lib = _lib.load()

    def sv(**kw):
        c = _lib.SamplerCfg()
        for k, v in kw.items():
            setattr(c, k, v)
        rc = lib.mcmc_sampler_validate(ct.byref(c))
        return rc, lib.mcmc_last_error().decode()

    assert sv(kind=1, scale=0.1)[0] == 0
    assert sv(kind=1, scale=0.0) == (1, "scale should be > 0")
    assert sv(kind=2, drift_step=-1.0) == (1, "MALA drift step should be > 0")
    assert sv(kind=3, n_leaps=0, leap_step=0.1) == (1, "inner steps should be > 0")
    assert sv(kind=3, n_leaps=2, leap_step=0.0) == (1, "inner steps scaling should be > 0")
    rc, msg = sv(kind=4, rate=1.5, len=2.0, shrinkage=0.05, t0=10.0, step=0.75)
    assert rc == 1 and msg.startswith("Target acceptance rate (1.5)")
    rc, msg = sv(kind=4, rate=0.65, len=2.0, shrinkage=0.0, t0=10.0, step=0.75)
    assert rc == 1 and "shrinkage parameter" in msg
    rc, msg = sv(kind=2, drift_step=0.1, tuner=1, adapt_step=0, max_step=10, target_rate=0.5)
    assert rc == 1 and msg.startswith("Adaptation step size (0)")

    def rv(b, t, n):
        c = _lib.RunnerCfg(b, t, n)
        return lib.mcmc_runner_validate(ct.byref(c)), lib.mcmc_last_error().decode()

    assert rv(100, 1, 1000)[0] == 0
    assert rv(-1, 1, 10) == (1, "Burnin rounds (-1) should be >= 0")
    assert rv(10, 1, 10) == (1, "Total MCMC length (10) should be > to burnin (10)")
    assert rv(0, 0, 10) == (1, "Thinning (0) should be >= 1")


def test_python_constructors_assert_like_reference():
    with pytest.raises(AssertionError, match="scale should be > 0"):
        mc.RWM(0.0)
    with pytest.raises(AssertionError, match="MALA drift step should be > 0"):
        mc.MALA(0.0)
    with pytest.raises(AssertionError, match="inner steps should be > 0"):
        mc.HMC(0, 0.1)
    with pytest.raises(AssertionError, match="Target acceptance rate"):
        mc.HMCDA(rate=1.0)
    with pytest.raises(AssertionError, match="Target acceptance rate"):
        mc.EmpMCTuner(1.5)
    h = mc.HMC(0.75)
    assert (h.nLeaps, h.leapStep) == (10, 0.75)                     # HMC(leapStep::Float64)
    h = mc.HMC(3)
    assert (h.nLeaps, h.leapStep) == (3, 0.1)                       # HMC(nLeaps::Int)
    h = mc.HMC(2, 0.1)
    assert (h.nLeaps, h.leapStep) == (2, 0.1)
    t = mc.EmpMCTuner(0.7)
    assert mc.MALA(t).tuner is t and mc.MALA(t).driftStep == 1.0  # MALA(s::MCMCTuner)
    da = mc.HMCDA()
    assert (da.rate, da.len, da.shrinkage, da.t0, da.step) == (0.65, 2.0, 0.05, 10.0, 0.75)


def test_model_semantics():
    m1 = mc.model(mc.IsoNormalDot(), init=np.ones(3))
    assert not m1.has_gradient and m1.size == 3 and (m1.scale == 1).all()
    m2 = mc.model(mc.IsoNormalDot(), grad=mc.IsoNormalDot.grad, init=np.ones(3))
    assert m2.has_gradient
    m = mc.model(mc.IsoNormalDot(), init=2.0, scale=0.5)             # scalar init/scale (likmodel.jl:112,115)
    assert m.size == 1 and m.init[0] == 2.0 and m.scale[0] == 0.5
    with pytest.raises(AssertionError, match="scale parameter size"):
        mc.model(mc.IsoNormalDot(), init=np.ones(3), scale=np.ones(2))
    # DSL packing: column-major, keyword order (expr_funcs.jl:76-90; test/dsl/unit_tests.jl:29-34)
    m = mc.model(mc.NormalDSL(), a=1.0, b=np.array([2.0, 3.0]), c=np.array([[4.0, 5.0], [6.0, 7.0]]))
    assert list(m.init) == [1.0, 2.0, 3.0, 4.0, 6.0, 5.0, 7.0]
    with pytest.raises(AssertionError, match="'init' kwargs not allowed"):
        mc.model(mc.NormalDSL(), init=np.ones(2), v=np.ones(2))


def test_needs_gradient_error():
    """run(mymodel3 * MALA(0.1) * SerialMC(1:1000)) throws (README.md:224, test_syntax.jl:75)."""
    m3 = mc.model(mc.NormalDSL(0, 1), v=np.ones(3))
    with pytest.raises(AssertionError, match="MALA sampler requires model with gradient function"):
        m3 * mc.MALA(0.1) * mc.SerialMC(range(1, 1001))
    with pytest.raises(AssertionError, match="HMC sampler requires model with gradient function"):
        m3 * mc.HMC(2, 0.1) * mc.SerialMC(steps=10)
    t = m3 * mc.RWM(0.1) * mc.SerialMC(steps=10)
    assert isinstance(t, mc.MCMCTask)


def test_star_composition_broadcasts():
    m = mc.model(mc.IsoNormalDot(), grad=True, init=np.ones(3))
    ts = m * [mc.RWM(0.1), mc.MALA(0.1), mc.HMC(3, 0.1)] * mc.SerialMC(steps=1000)
    assert len(ts) == 3 and [type(t.sampler).__name__ for t in ts] == ["RWM", "MALA", "HMC"]
    ts = m * [mc.HMC(i, 0.1) for i in range(1, 6)] * mc.SerialMC(steps=1000)
    assert [t.sampler.nLeaps for t in ts] == [1, 2, 3, 4, 5]


def test_no_gpu_means_loud_failure():
    if mc.device_count() > 0:
        pytest.skip("a GPU is present")
    m = mc.model(mc.IsoNormalDot(), init=np.ones(3))
    with pytest.raises(mc.MCMCError):
        mc.run(m * mc.RWM(0.1) * mc.SerialMC(steps=10))


def test_accept_bit_unpacking():
    from mcmchip.api import _unpack_bits
    C = 130
    rng = np.random.default_rng(0)
    acc = rng.random((4, C)) < 0.5
    words = np.zeros((4, 3), dtype=np.uint64)
    for k in range(4):
        for c in range(C):
            if acc[k, c]:
                words[k, c // 64] |= np.uint64(1) << np.uint64(c % 64)
    assert np.array_equal(_unpack_bits(words, C), acc.T)


def test_store_leaps_options():
    """storeLeaps (HMC.jl:145-150, HMCDA.jl:110-117) is accepted; the record keeps nLeaps (or the tuner's maxStep,
    or HMCDA's max_leaps) states per kept step"""
    assert mc.HMC(4, 0.3, storeLeaps=True).leaps_cap() == 4
    assert mc.HMC(3, 0.9, mc.EmpMCTuner(0.7, maxStep=9), storeLeaps=True).leaps_cap() == 9
    assert mc.HMCDA(storeLeaps=True, max_leaps=40).leaps_cap() == 40
    assert mc.HMCDA(storeLeaps=True).leaps_cap() == 256
    assert not mc.HMC().storeLeaps


def test_bench_traffic_only_from_a_profile_of_the_same_kernel():
    """bench.py fills roofline.traffic from profiles/traffic.json only when the committed profile is of the same
    workload AND the same step kernel instance (a profile of another kernel is stale)"""
    import importlib
    import json
    bench = importlib.import_module("bench")
    t = json.load(open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "profiles", "traffic.json")))
    for key in t:
        assert bench.measured_traffic(key, t[key]["kernel"])["bytes_per_launch"] == t[key]["traffic_bytes"]
        assert bench.measured_traffic(key, "glm_mala<8,1>") is None
        assert os.path.exists(os.path.join(ROOT, t[key]["source"]))
    assert bench.measured_traffic("no-such-workload", "lpc_rwm") is None
    # the driver's exact command (bench.py --gpus 1 --steps 20 --warmup 5) has a committed profile
    dkey = "metric|d=32|chains=1048576|rwm|steps=20|thinning=10|spl=0"
    assert bench.measured_traffic(dkey, "lpp_rwm<4, true, IsoDot, true>") is not None     # two lanes per chain
    assert bench.measured_traffic(dkey, "lpp_rwm<4, true, IsoDot, false>") is None


def test_bench_valu_roofline_profile():
    """A VALU profile prices a run only when it was recorded from the sources of its kernel's family (the regression
    kernels' or the other step kernels'), for the same kernel instance and the same workload (steps included); every
    committed profile implies a VALU fraction <= 1 at its own measured clock."""
    import importlib
    import json
    bench = importlib.import_module("bench")
    prof = json.load(open(os.path.join(ROOT, "profiles", "valu.json")))
    assert bench.kernel_src_hash("glm_rwm<1, 1>") == bench.glm_src_hash()
    assert bench.kernel_src_hash("void mcmc::lpp_rwm<4, true, IsoDot, true>(mcmc::KernelArgs)") == bench.step_kernel_src_hash()
    for k, e in prof.items():
        got = bench.measured_valu(e["kernel"], e["workload_key"])
        assert (got is not None) == (e["src_hash"] == bench.kernel_src_hash(e["kernel"]))
        assert bench.measured_valu(e["kernel"], e["workload_key"] + "x") is None      # another workload
        assert bench.measured_valu("lpc_rwm<9,true,X,true>", e["workload_key"]) is None
        assert os.path.exists(os.path.join(ROOT, e["source"]))
        assert 0.0 < e["valu_busy"] <= 1.0
        steps = int(e["workload_key"].split("steps=")[1].split("|")[0])
        chains = int(e["workload_key"].split("chains=")[1].split("|")[0])
        cyc = 4 * e["valu_quadcycles_per_chain_step"] * chains * steps       # VALU issue cycles of the launch
        frac_at_clock = cyc / e["duration_s"] / (1024 * e["clock_ghz"] * 1e9)
        assert 0.3 < frac_at_clock <= 1.0 + 1e-6, (k, frac_at_clock)


def _c_struct_fields(name):
    """(field, julia type) of a typedef struct in include/mcmc_hip.h, in order."""
    import re
    h = open(os.path.join(ROOT, "include", "mcmc_hip.h")).read()
    body = re.search(r"typedef struct \{([^{}]*)\}\s*" + name + ";", h).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    ty = {"int32_t": "Int32", "int64_t": "Int64", "double": "Float64", "double*": "Ptr{Float64}",
          "uint64_t*": "Ptr{UInt64}"}
    out = []
    for decl in body.split(";"):
        decl = decl.replace("const ", "").strip()
        if not decl:
            continue
        m = re.match(r"(\w+\s*\*?)\s*(.*)", decl)
        base = m.group(1).replace(" ", "")
        for nm in m.group(2).split(","):
            nm = nm.strip()
            t = base
            if nm.startswith("*"):
                nm, t = nm[1:].strip(), base + "*"
            out.append((nm, ty[t]))
    return out


def _jl_struct_fields(path, jname):
    import re
    s = open(path).read()
    body = re.search(r"(?:immutable|type|struct|mutable struct)\s+" + jname + r"\b(.*?)\bend\b", s,
                     flags=re.S).group(1)
    body = re.sub(r"#[^\n]*", "", body)
    fields = []
    for part in re.split(r"[;\n]", body):
        part = part.strip()
        if part:
            nm, t = part.split("::")
            fields.append((nm.strip(), t.strip().replace("Uint64", "UInt64")))
    return fields


@pytest.mark.parametrize("c_name,hook_name,plain_name", [
    ("mcmc_model_desc", "HipModelDesc", "ModelDesc"), ("mcmc_sampler_cfg", "HipSamplerCfg", "SamplerCfg"),
    ("mcmc_runner_cfg", "HipRunnerCfg", "RunnerCfg"), ("mcmc_outputs", "HipOutputs", "Outputs")])
def test_julia_hook_structs_mirror_header(c_name, hook_name, plain_name):
    """Both Julia bindings (the MCMC.jl hook for the reference's Julia, MCMCHip.jl for Julia >= 1.0) declare the
    C structs field for field: same names, order and types (there is no Julia in the image to compile them)."""
    jdir = os.path.join(ROOT, "mcmc.jl_amd", "julia")
    c = _c_struct_fields(c_name)
    assert _jl_struct_fields(os.path.join(jdir, "mcmc_jl_hook.jl"), hook_name) == c
    assert _jl_struct_fields(os.path.join(jdir, "MCMCHip.jl"), plain_name) == c


def test_julia_hook_defines_batched_runners_reset_ou_and_leaps():
    """The MCMC.jl hook (Julia 0.3 text, no Julia here): run(::Array{MCMCTask}) and prun(::Array{MCMCTask}) are
    redefined with the batched GPU path and the reference's dispatch as fallback (runners.jl:17-42), every GPU task
    installs the :reset hook MCMC.reset calls (MCMC.jl:39), the OU model kind is there, storeLeaps records map into
    diagnostics["leaps"] as HMCSample arrays, and spun tasks draw their chains from the global stream rather than a
    fixed seed."""
    jl = open(os.path.join(ROOT, "mcmc.jl_amd", "julia", "mcmc_jl_hook.jl")).read()
    for needle in ("function run(t::Array{MCMCTask}; args...)", "function prun(t::Array{MCMCTask}; args...)",
                   "hip_batchable(t) && return hip_run_tasks(t, false)",
                   "hip_batchable(t) && return hip_run_tasks(t, true, hip_devices())",
                   "run_seqmc(t; args...)", "pmap(run_serialmc_exit, t)", "run_serialtempmc(t)",
                   "task_local_storage(:reset,", ":ou => 9", "mcmc_chains_fork", "mcmc_chains_set_state",
                   'diag["leaps"] = hip_leap_states', 'diags["leaps"]', "HMCSample(", "mcmc_chains_store_leaps",
                   "hip_draw(1)", "hip_srand", "stop!(res[k])"):
        assert needle in jl, needle
    assert "seed = 1\n" not in jl                       # no fixed per-task seed
    plain = open(os.path.join(ROOT, "mcmc.jl_amd", "julia", "MCMCHip.jl")).read()
    for needle in ("function ou_model", "MODEL_OU", "mcmc_chains_set_state", "mcmc_chains_fork"):
        assert needle in plain, needle


def test_julia_hook_runner_semantics():
    """The hook's runner semantics, as text (no Julia here; tests/test_hook_protocol.py drives the
    same C calls on the GPU): every task sets its runner's burnin as the tuners' burnin on its chains (fresh and
    forked), chunks are at most the task runner's len, the tasks of one model share one uploaded model, prun of like
    GPU tasks runs one mcmc_group over every visible device, SeqMC arrays of GPU targets go to mcmc_run_seqmc, drawn
    streams use their own key space, and the ESS of a GPU batch is one mcmc_stats_ess call."""
    import re
    jl = open(os.path.join(ROOT, "mcmc.jl_amd", "julia", "mcmc_jl_hook.jl")).read()
    ens = jl[jl.index("function hip_ensure!"):jl.index("end", jl.index("hip_set_tuner_burnin!(st.chains"))]
    assert ens.index("HipChains(st.src, st.first, 1)") < ens.index("hip_set_tuner_burnin!(st.chains, "
                                                                     "hip_tuner_burnin(st.runner))")
    assert "hip_tuner_burnin(r::MCMCRunner) = (isa(r, SerialMC) || isa(r, SeqMC)) ? r.burnin : 0" in jl
    assert "ccall((:mcmc_chains_set_tuner_burnin, hiplib), Cint, (Ptr{Void}, Int64)" in jl
    assert "n = isa(st.runner, SerialMC) ? min(hip_chunk, st.runner.len) : 1" in jl
    assert "HipTaskState(m, s, r)" in jl and "HipModelHandle(hip_context(m.device), m)" in jl
    assert jl.count("HipModelHandle(") == 2            # its inner constructor and the one cached construction
    assert "hip_batchable(t) && return hip_run_tasks(t, true, hip_devices())" in jl
    for sym in ("mcmc_group_create", "mcmc_group_chains_create", "mcmc_group_run_serialmc",
                "mcmc_group_chains_destroy", "mcmc_device_count", "mcmc_run_seqmc", "mcmc_stats_ess"):
        assert f"ccall((:{sym}, hiplib)" in jl, sym
    assert "isa(lastrunner, SeqMC) && hip_seqmc_able(t) && return hip_run_seqmc(t; args...)" in jl
    assert "function ess(cs::Array{MCMCChain}" in jl
    assert "hip_key(seed::Int) = (uint64(seed) & 0x7fffffffffffffff) | 0x8000000000000000" in jl
    # every library function the hook calls is declared in the header
    hdr = open(os.path.join(ROOT, "include", "mcmc_hip.h")).read()
    for sym in set(re.findall(r"ccall\(\(:(\w+), hiplib\)", jl)):
        assert re.search(r"\b" + sym + r"\(", hdr), sym


def test_spun_tasks_draw_from_the_global_stream():
    """m * s * r tasks carry no stream until they run; srand restarts the cursor; draws are consecutive and move to
    the next key before the 32-bit chain id would overflow; explicit seeds keep offset 0 (host logic only)."""
    from mcmchip import api
    m = mc.model(mc.IsoNormalDot(), init=np.ones(3), grad=True)
    r = mc.SerialMC(steps=10)
    t = m * mc.RWM(0.1) * r
    assert t.seed is None and t.chain_offset is None
    ts = m * [mc.RWM(0.1), mc.RWM(0.1)] * r
    assert all(x.seed is None for x in ts) and api._same_task_kind(ts[1], ts[0])
    assert not api._same_task_kind((m * mc.MALA(0.1) * r), ts[0])
    assert not api._same_task_kind((m * mc.RWM(0.2) * r), ts[0])
    mc.srand(5)
    assert api._draw_chains(3) == (api.drawn_key(5), 0) and api._draw_chains(2) == (api.drawn_key(5), 3)
    api._GlobalStream.next_chain = (1 << 32) - 1
    assert api._draw_chains(2) == (api.drawn_key(6), 0)
    mc.srand(9)
    b = t.batch(64)
    assert b.seed is None and b.chain_offset is None
    b._draw()
    assert (b.seed, b.chain_offset) == (api.drawn_key(9), 0) and api._GlobalStream.next_chain == 64
    e = t.batch(64, seed=3)
    assert (e.seed, e.chain_offset) == (3, 0)
    with pytest.raises(ValueError):
        mc.MCMCTask(m, mc.RWM(0.1), r, seed=None, chain_offset=4)
    # drawn streams have their own key space: no explicit seed (< 2^63) names a drawn stream
    assert api.drawn_key(1) == (1 << 63) | 1 and api.drawn_key(1) != 1 and api.drawn_key(api.drawn_key(3)) == api.drawn_key(3)
    from mcmchip.seqmc import target_seed
    assert all(target_seed(s, k) < 1 << 63 for s in (1, 2**63 - 1, 12345) for k in range(5))


def test_prun_dispatch_devices(monkeypatch):
    """prun of like tasks: one group over every visible GPU, except storeLeaps samplers, whose records are built for
    one device (host logic only: the batch runner is stubbed)."""
    from mcmchip import api
    seen = []
    monkeypatch.setattr(api, "device_count", lambda: 4)
    monkeypatch.setattr(api, "_run_batched", lambda ts, stop=False, devices=None: seen.append((stop, devices)) or [])
    m = mc.model(mc.IsoNormalDot(), init=np.ones(3), grad=True)
    r = mc.SerialMC(steps=10)
    mc.prun(m * [mc.HMC(3, 0.1), mc.HMC(3, 0.1)] * r)
    mc.prun(m * [mc.HMC(3, 0.1, storeLeaps=True), mc.HMC(3, 0.1, storeLeaps=True)] * r)
    mc.prun(m * [mc.RWM(0.1)] * r, devices=(1, 2))
    assert seen == [(True, (0, 1, 2, 3)), (True, None), (True, (1, 2))]
