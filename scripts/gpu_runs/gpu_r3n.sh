# round 3: VALU PMC of config 2 and config 4 at the bench defaults (profiles keyed by workload), metric20 line
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 600 bash scripts/gpu_pmc.sh r3n_d3 --config d3 --no-ess > $O/pmcd3.log 2>&1 || exit 1
timeout -k 10 900 bash scripts/gpu_pmc.sh r3n_hmc1024 --config hmc1024 --no-ess > $O/pmch.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/gpu_prof.sh r3n_d3 --config d3 --no-ess > $O/profd3.log 2>&1 || exit 1
timeout -k 10 900 bash scripts/gpu_prof.sh r3n_hmc1024 --config hmc1024 --no-ess > $O/profh.log 2>&1 || exit 1
echo all-done
