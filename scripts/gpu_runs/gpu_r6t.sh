# round 6 final build: the bench sweep (defaults, cpu_baseline on), after the PMC profiles it reads
# (profiles/valu.json, fp64.json, traffic.json), so every line names its binding resource.  PART=sep | glm
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
if [ "${PART:-sep}" = sep ]; then
  run driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
  run metric 300 python3 bench.py
  for c in readme d3 hmc1024 bare_normal ram32 ram256; do run $c 300 python3 bench.py --config $c; done
  run mala32 300 python3 bench.py --sampler mala --no-cpu-baseline --no-ess
  run hmc32 300 python3 bench.py --sampler hmc --no-cpu-baseline --no-ess
else
  for c in logistic128 linear512 linear1024 ramlinear128 binomial ramlinear; do run $c 400 python3 bench.py --config $c; done
fi
echo all-done
