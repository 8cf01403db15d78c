# round 5: the pair RWM kernel's next-block state prefetch (PairChain::prefetch_state): GPU suite on the new build,
# then A/B against the same sources built with -DMCMC_STATE_PREFETCH=0, alternating on one box
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
L=mcmc.jl_amd/mcmchip
run gputests 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for rep in 1 2 3; do
  for v in base nopf; do
    if [ $v = base ]; then lib=$L/libmcmc_hip.so; else lib=$L/libmcmc_hip_$v.so; fi
    MCMCHIP_LIB=$lib run metric20_${v}_$rep 200 python3 bench.py --steps 20 --warmup 5 --no-ess --no-cpu-baseline
  done
done
for v in base nopf; do
  if [ $v = base ]; then lib=$L/libmcmc_hip.so; else lib=$L/libmcmc_hip_$v.so; fi
  MCMCHIP_LIB=$lib run metric1000_${v} 200 python3 bench.py --steps 1000 --warmup 5 --no-ess --no-cpu-baseline
done
echo all-done
