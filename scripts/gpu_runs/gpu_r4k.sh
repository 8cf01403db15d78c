# round 4: wave RAM with row-interleaved factor ownership (coalesced column accesses, LDS layout changes of z and
# S z): RAM parity + ram256; then the driver's metric command (20 steps, warmup 5) bench, VALU PMC and traffic
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run tests 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_group.py -m gpu -x -q -k "ram_ or _ram or ou_" --timeout 300 --timeout-method thread
run ram256 300 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
run metric20 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run pmc_m20 400 bash scripts/gpu_pmc.sh r4k_metric20 --steps 20 --warmup 5 --no-ess
run prof_m20 400 bash scripts/gpu_prof.sh r4k_metric20 --steps 20 --warmup 5 --no-ess
echo all-done
