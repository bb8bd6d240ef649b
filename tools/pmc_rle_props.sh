#!/bin/bash
# Counters of the RLE family alone on the property plan (OPB_PROPS=1 tools/family_run.py rle): instruction
# mix, memory pipeline and L2 request counts, one rocprofv3 --pmc pass per counter set.
#   tools/pmc_rle_props.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp OPB_PROPS=1
O=${1:-gpurun_out/pmc_rle_props}
mkdir -p "$O"
SETS=("GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES"
      "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU"
      "GRBM_GUI_ACTIVE TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCC_WRITE_REQ_sum TD_TD_BUSY TD_TC_STALL"
      "GRBM_GUI_ACTIVE TCC_REQ_sum TCC_WRITE_sum SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS")
i=0
for s in "${SETS[@]}"; do
    timeout -s KILL 90 rocprofv3 --pmc $s -d "$O/p$i" -o run --output-format csv -- \
        python tools/family_run.py rle 2 > "$O/p$i.log" 2>&1 || echo "pass $i failed"
    i=$((i + 1))
done
python tools/pmc_summary.py "$O/*/run_counter_collection.csv" > "$O/summary.txt" 2>&1 || true
echo done
