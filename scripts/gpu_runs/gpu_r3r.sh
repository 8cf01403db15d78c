# round 3: where the 20-step launch's fixed cost goes (kept-row stores vs state I/O vs rounds)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3r
mkdir -p $O
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --thinning 1000" "--steps 40 --warmup 5" "--steps 40 --warmup 5 --thinning 1000" "--steps 20 --warmup 5 --chains 524288" "--steps 2 --warmup 5 --thinning 1000" "--steps 100 --warmup 5"; do
  n=$(echo $args | tr -d ' -')
  timeout -k 10 240 python bench.py $args --no-cpu-baseline --no-ess > $O/b_$n.json 2> $O/b_$n.err || exit 1
done
echo all-done
