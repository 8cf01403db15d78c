# round 4: d-sliced glm_eval with asm LDS-DMA, hoisted operand reads, [wave][r][lane] partials: parity + config 5
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run glmtests 600 python3 -u -m pytest tests -m gpu -x -q -k "glm or config3 or config5 or golden or store_leaps or logistic or group" --timeout 300 --timeout-method thread
run lin512 300 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run lin256 300 python3 bench.py --config linear512 --d 256 --no-cpu-baseline --no-ess
echo all-done
