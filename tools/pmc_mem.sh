#!/bin/bash
# Memory-pipeline counters (TA / TD / TCP) of the config-5 launch and of each family alone, one
# rocprofv3 --pmc pass per counter set and target (tools/family_run.py), plus the box's counter list.
#   tools/pmc_mem.sh OUTDIR
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_mem}
mkdir -p "$O"
timeout -s KILL 60 rocprofv3 -L > "$O/counters_list.txt" 2>&1 || true
SETS=("GRBM_GUI_ACTIVE TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES"
      "GRBM_GUI_ACTIVE TD_TD_BUSY TD_TC_STALL SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU")
for fam in all fastpfor varint rle; do
    i=0
    for s in "${SETS[@]}"; do
        timeout -s KILL 90 rocprofv3 --pmc $s -d "$O/${fam}_$i" -o run --output-format csv -- \
            python tools/family_run.py $fam 2 > "$O/${fam}_$i.log" 2>&1 || echo "pass ${fam}_$i failed"
        i=$((i + 1))
    done
done
python tools/pmc_summary.py "$O/*/run_counter_collection.csv" > "$O/summary.txt" 2>&1 || true
echo done
