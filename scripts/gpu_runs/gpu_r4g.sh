# round 4: y = x * v; y ~ D (bare_distribs.jl) parity + bench line; then r4f's stamps and DMA-spread A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run tests 600 python3 -u -m pytest tests -m gpu -q -k "dist_obs" --timeout 300 --timeout-method thread
run bare 300 python3 bench.py --config bare_normal --no-ess
bash scripts/gpu_runs/gpu_r4f.sh
