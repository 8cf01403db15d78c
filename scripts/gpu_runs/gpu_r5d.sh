# round 5: A/B of the config-3 kernel's eta operand look-ahead (4 / 8 / 12), alternating libraries on one box; the
# widened regression sizes' bench lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
L=mcmc.jl_amd/mcmchip
for rep in 1 2; do
  for v in base la8 la12; do
    if [ $v = base ]; then lib=$L/libmcmc_hip.so; else lib=$L/libmcmc_hip_$v.so; fi
    MCMCHIP_LIB=$lib run log128_${v}_$rep 200 python3 bench.py --config logistic128 --steps 20 --warmup 2 --no-ess --no-cpu-baseline
  done
done
run lin1024 600 python3 bench.py --config linear1024 --no-cpu-baseline --no-ess
run ramlin128 300 python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess
echo all-done
