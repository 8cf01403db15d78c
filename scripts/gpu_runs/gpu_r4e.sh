# round 4: probit model (erfc / erfcx / normal log-cdf on the device) parity, detmath ops 18-21, GLM parity; then the
# d-sliced tile-loop phase stamps (GLM_STAMP build)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run tests 900 python3 -u -m pytest tests -m gpu -q -k "probit or detmath or glm or config3 or config5" --timeout 300 --timeout-method thread
run st512 300 env MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_stamp.so python3 scripts/glm_stamps.py 512 4096 8192
run st256 300 env MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_stamp.so python3 scripts/glm_stamps.py 256 4096 8192
echo all-done
