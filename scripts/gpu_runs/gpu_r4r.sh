# round 4 sweep of the other bench configs on the final build (default arguments, cpu_baseline on), the metric's
# MALA / HMC shapes, and the VALU PMC of the 1 000-step metric, d3 and hmc1024 for the final sources
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
for c in readme d3 hmc1024 binomial bare_normal ram32 ram256 ramlinear; do run $c 300 python3 bench.py --config $c --no-ess; done
run mala32 300 python3 bench.py --sampler mala --no-cpu-baseline --no-ess
run hmc32 300 python3 bench.py --sampler hmc --no-cpu-baseline --no-ess
run pmc_m1000 300 bash scripts/gpu_pmc.sh r4r_metric1000 --steps 1000 --no-ess
run pmc_d3 300 bash scripts/gpu_pmc.sh r4r_d3 --config d3 --no-ess
run pmc_hmc1024 300 bash scripts/gpu_pmc.sh r4r_hmc1024 --config hmc1024 --no-ess
echo all-done
