# round 3: LDS Box-Muller tables for lane-per-chain MALA / HMC / RAM (RAM d=32 regressed 2.7x with global tables)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config ram32 --no-cpu-baseline > $O/bench_ram32.json 2> $O/bench_ram32.err || exit 1
for d in 4 8 16; do for sm in mala hmc; do
timeout -k 10 300 python bench.py --d $d --sampler $sm --steps 200 --warmup 20 --no-cpu-baseline --no-ess > $O/bench_${sm}_d$d.json 2> $O/bench_${sm}_d$d.err || exit 1
done; done
echo all-done
