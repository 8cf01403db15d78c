# round 4: staged-tile X image + LDS-DMA + 128-wide d-slices: regression parity, then configs 5 / 3 / binomial.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run lin512n 300 env MCMCHIP_GLM_SLICE=64 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run log128 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
run glmtests 600 python3 -u -m pytest tests -m gpu -q -k "glm or config3 or config5 or golden or store_leaps or logistic" --timeout 300 --timeout-method thread
echo all-done
