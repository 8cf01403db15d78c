# round 2, session 4: register-resident ESS kernel (k_ess_reg) -- bitwise ESS tests, metric-shape timing, and the
# fp64 MFMA / VALU co-execution probe (scripts/peak_f64.hip).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4c_tests 300 python3 -u -m pytest tests -m gpu -k "ess" -x -q --timeout 120 --timeout-method thread
run s4c_probe 300 python3 scripts/ess_probe.py
run s4c_peak 120 scripts/_build/peak_f64
echo all-done
