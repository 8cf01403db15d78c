# PMC passes (one counter group per pass, --kernel-trace only) for a bench config.
# usage: bash scripts/gpu_pmc.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/pmc_$tag
mkdir -p "$O"
rocprofv3 -L > "$O/counters_list.txt" 2>&1 || true
i=0
PGROUPS=${PMC_GROUPS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64;SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES"}
IFS=';' read -ra GRPS <<< "$PGROUPS"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$O/p$i" -o run -- python3 bench.py --no-cpu-baseline "$@" > "$O/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc $rc" | tee -a "$O/steps.txt"
  case $rc in 0|1) ;; *) echo "stopping (rc $rc)"; exit $rc;; esac
done
echo pmc-done
