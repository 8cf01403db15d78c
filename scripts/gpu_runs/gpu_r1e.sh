cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name exit $rc" | tee -a "$O/steps.txt"
  case $rc in 0|1|2|5) return 0;; *) echo "fatal rc $rc in $name: stopping"; exit $rc;; esac
}
step r1e_glm 900 python3 -m pytest tests/test_gpu_parity.py -q -k "glm or logistic" --maxfail=5
step r1e_all 900 python3 -m pytest tests -q -m gpu --maxfail=5
echo all-done
