# round 6, call AQ: RAM on regression targets with the two halves staggered (the second half's first eval after the
# first half's), against both halves starting at once (MCMCHIP_RAM_STAGGER=0); parity of the split step first
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6aq
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_bench_instances.py -m gpu -x -q -k "ram" --timeout 120 --timeout-method thread -p no:cacheprovider
B="python3 bench.py --config ramlinear128 --no-cpu-baseline --no-ess"
run stg 300 $B
MCMCHIP_RAM_STAGGER=0 run nostg 300 $B
run stg2 300 $B
MCMCHIP_RAM_STAGGER=0 run nostg2 300 $B
echo all-done
