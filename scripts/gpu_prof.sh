# rocprofv3 summaries for the bench workload: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE passes.
# usage: bash scripts/gpu_prof.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/prof_$tag
mkdir -p "$O"
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name exit $rc" | tee -a "$O/steps.txt"
  [ $rc -eq 0 ] || { echo "stopping after $name (rc $rc)"; exit $rc; }
}
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 bench.py --no-cpu-baseline "$@"
run fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- python3 bench.py --no-cpu-baseline "$@"
run write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- python3 bench.py --no-cpu-baseline "$@"
echo prof-done
