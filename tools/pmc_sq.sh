mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq -o run --output-format csv -- python tools/family_run.py all 2 > gpurun_out/pmc_sq.log 2>&1
echo rc=$?
