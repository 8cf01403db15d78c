# round 5: A/B experiments, alternating libraries on one box: the metric kernel as a persistent grid (LPP_PERSIST),
# config 3 with a two-accumulator eta chain (GLM_WS_ETA2; not bitwise: timing only)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
L=mcmc.jl_amd/mcmchip
for rep in 1 2; do
  for v in base persist; do
    if [ $v = base ]; then lib=$L/libmcmc_hip.so; else lib=$L/libmcmc_hip_$v.so; fi
    MCMCHIP_LIB=$lib run metric20_${v}_$rep 200 python3 bench.py --steps 20 --warmup 5 --no-ess --no-cpu-baseline
    MCMCHIP_LIB=$lib run metric200_${v}_$rep 200 python3 bench.py --steps 200 --warmup 5 --no-ess --no-cpu-baseline
  done
  for v in base eta2; do
    if [ $v = base ]; then lib=$L/libmcmc_hip.so; else lib=$L/libmcmc_hip_$v.so; fi
    MCMCHIP_LIB=$lib run log128_${v}_$rep 200 python3 bench.py --config logistic128 --steps 20 --warmup 2 --no-ess --no-cpu-baseline
  done
done
echo all-done
