# round 5: full GPU suite on the stream / fork / reset boundary work, then the driver's bench line and configs 3 / 5
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run gputests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
run bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
run lin512 400 python3 bench.py --config linear512 --no-cpu-baseline --no-ess
run log128 300 python3 bench.py --config logistic128 --no-cpu-baseline --no-ess
echo all-done
