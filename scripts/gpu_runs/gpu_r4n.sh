# round 4 final check: the driver's bench command, its VALU PMC + traffic profiles for the final sources (pair-kernel
# stores recompute the chain index: no scratch), the whole GPU suite, smoke()
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run bench0 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess
run pmc_m20 400 bash scripts/gpu_pmc.sh r4n_metric20 --steps 20 --warmup 5 --no-ess
run prof_m20 400 bash scripts/gpu_prof.sh r4n_metric20 --steps 20 --warmup 5 --no-ess
run tests 1100 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo all-done
