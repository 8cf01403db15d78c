# round 2, session 4: k_ess_reg Markstein quotients + zero-pad block skip -- ESS tests, timing, PMC; fp64 fma latency probe.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run s4e_tests 300 python3 -u -m pytest tests -m gpu -k "ess" -x -q --timeout 120 --timeout-method thread
run s4e_probe 300 python3 scripts/ess_probe.py
run s4e_pmc1 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/s4e_pmc1 -o run -- python3 scripts/ess_probe.py
echo all-done
