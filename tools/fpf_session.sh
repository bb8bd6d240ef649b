#!/bin/bash
# FastPFOR A/B session: GPU tests, paired timing (tools/ab.py) and per-family utilisation counters for the
# base and the new library (each --pmc pass its own run).  usage: tools/fpf_session.sh [variants...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${*:-libcovt_base.so libcovt.so}
bash tools/gpu_session.sh tests || exit $?
AB_VARIANTS="$V" bash tools/gpu_session.sh abfpf || exit $?
for v in $V; do
    n=${v%.so}
    COVT_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/util_$n -o run --output-format csv -- python tools/family_run.py fastpfor 2 > gpurun_out/util_$n.log 2>&1 || exit $?
    COVT_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/wait_$n -o run --output-format csv -- python tools/family_run.py fastpfor 2 > gpurun_out/wait_$n.log 2>&1 || exit $?
    COVT_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/inst_$n -o run --output-format csv -- python tools/family_run.py fastpfor 2 > gpurun_out/inst_$n.log 2>&1 || exit $?
done
echo "fpf session done"
