# round 4: opaque lane pointers (no hoisted per-slot addresses: the d-sliced regression kernels stop spilling), HMC
# momentum parked in HBM across evaluations, the metric kernel's exact log test out of line.  GLM + metric parity;
# config 5 at 64- and 128-wide d-slices, d = 256 likewise; RAM two chains per wave (d <= 256) parity + ram256;
# the driver's metric command
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run tests 900 python3 -u -m pytest tests -m gpu -x -q -k "glm or config or probit or golden or screened or detmath or store_leaps or metric or readme or ram" --timeout 300 --timeout-method thread
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run lin512w 300 env MCMCHIP_GLM_SLICE=128 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run lin256 300 python3 bench.py --config linear512 --d 256 --no-cpu-baseline --no-ess
run lin256w 300 env MCMCHIP_GLM_SLICE=128 python3 bench.py --config linear512 --d 256 --no-cpu-baseline --no-ess
run ram256 300 python3 bench.py --config ram256 --no-cpu-baseline --no-ess
run metric20 300 python3 bench.py --no-cpu-baseline --no-ess
echo all-done
