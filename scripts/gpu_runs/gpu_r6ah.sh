# round 6, call AH (final sources: tile skip + pairing): the tile-pairing parity test, then the regression part of
# the bench sweep (defaults, cpu_baseline on) after the r6ag PMC profiles it reads
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ah
mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || exit $rc; }
run pairtest 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "tile_pairing or trajectory_order" --timeout 120 --timeout-method thread -p no:cacheprovider
for c in logistic128 linear512 linear1024 ramlinear128 binomial ramlinear; do run $c 400 python3 bench.py --config $c; done
echo all-done
