# round 2 session 4: every BASELINE config on the current build (bench.py defaults per config; CPU baseline on the
# box's host cores), for DESIGN.md §7's table.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4o_metric 300 python3 bench.py
run s4o_readme 200 python3 bench.py --config readme
run s4o_d3 300 python3 bench.py --config d3
run s4o_log 300 python3 bench.py --config logistic128
run s4o_hmc 400 python3 bench.py --config hmc1024
run s4o_lin 300 python3 bench.py --config linear512
run s4o_ram 300 python3 bench.py --config ram32 --no-cpu-baseline
run s4o_ramlin 300 python3 bench.py --config ramlinear --no-cpu-baseline
echo all-done
