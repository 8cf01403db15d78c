# round 4: 128-wide d-slices default for 256 < d <= 512 (config 5 glm_hmc<8, 4, true>); wave RAM with range-checked
# unconditional buffer accesses (exact vmcnt waits); GLM / RAM / OU parity, config 5 and ram256 benches
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run tests 900 python3 -u -m pytest tests -m gpu -x -q -k "glm or config or probit or golden or ram_ or _ram or ou_ or store_leaps or group" --timeout 300 --timeout-method thread
run ram256 300 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run log128 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
echo all-done
