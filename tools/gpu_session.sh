#!/bin/bash
# Runs GPU steps in sequence on the gpurun box.  Every step has its own time limit; an abort,
# segfault, time limit or GPU fault ends the session (no further GPU step runs).  Plain test
# failures (pytest rc 1) do not.
# usage: tools/gpu_session.sh STEP...   where STEP is one of: tests smoke bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "FATAL step=$1 rc=$2"; exit "$2"; }
step() {  # step NAME LIMIT cmd...
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 5 "gpurun_out/$name.log"
    if grep -q -E "Memory access fault|HSA_STATUS_ERROR|hipErrorIllegalAddress|GPU Hang" "gpurun_out/$name.log"; then fatal "$name" 99; fi
    case $rc in 0|1|5) ;; *) fatal "$name" "$rc";; esac
}
for s in "$@"; do
    # STEP+props: the same step on the property plan (OPB_PROPS=1), logs suffixed _props
    unset OPB_PROPS; sfx=
    case $s in *+props) export OPB_PROPS=1; sfx=_props; s=${s%+props};; esac
    case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    abfpf) step ab_fpf 900 python tools/ab.py ${AB_VARIANTS:-libcovt_base.so libcovt.so} ;;
    tests_asm) step pytest_gpu_asm 600 python -m pytest tests/test_gpu_assembly.py -m gpu -q -p no:cacheprovider --durations=5 ;;
    asm_ab) for v in ${AB_VARIANTS:-libcovt_asm1.so libcovt_asm2.so libcovt_asm3.so libcovt.so libcovt_asm1.so libcovt_asm2.so libcovt_asm3.so libcovt.so}; do
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/asm_run.py 20 2>&1 | grep -v amdgpu.ids || fatal asm_ab $?
        done ;;
    pmc_asm) step pmc_asm_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_asm_fetch -o run --output-format csv -- python tools/asm_run.py 3 && \
             step pmc_asm_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_asm_write -o run --output-format csv -- python tools/asm_run.py 3 ;;
    sq_asm) step sq_asm 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/sq_asm -o run --output-format csv -- python tools/asm_run.py 3 && \
            step mem_asm 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d gpurun_out/mem_asm -o run --output-format csv -- python tools/asm_run.py 3 ;;
    asm_longpole) step asm_longpole 300 python tools/asm_longpole.py 10 ;;
    asm_debug) step asm_debug 300 python tools/asm_debug.py 1 ;;
    tests_all) step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    bench_short) step bench 600 python bench.py --steps 10 --warmup 3 --cpu-iters 3 ;;
    ops) step op_breakdown 600 python tools/op_breakdown.py ;;
    timeline) step timeline 300 python tools/stream_timeline.py ;;
    timeline_props) step timeline_props 300 python tools/stream_timeline.py --props ;;
    hbm) step hbm 300 python tools/hbm_probe.py ;;
    wpat) step wpat 300 python tools/probe/write_pattern.py ;;
    ceiling) step ceiling 300 python tools/probe/hbm_ceiling.py ;;
    layout) step layout 300 python tools/probe/layout_ab.py ;;
    ab|ab_props) [ "$s" = ab_props ] && export OPB_PROPS=1
        for v in ${AB_VARIANTS:-libcovt_base.so libcovt.so libcovt_base.so libcovt.so}; do
            echo "== ab $v"; COVT_LIB_VARIANT=$v OPB_QUICK=1 timeout -k 10 300 python tools/op_breakdown.py 2>&1 | grep -v amdgpu.ids || fatal ab $?
        done ;;
    props_ab) for v in ${AB_VARIANTS:-libcovt_base.so libcovt.so libcovt_base.so libcovt.so}; do
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/props_run.py 2>&1 | grep -v amdgpu.ids || fatal props_ab $?
        done ;;
    timeline_omt) step timeline_omt 300 python tools/stream_timeline.py 9000 --omt ;;
    asm_props_ab) for v in ${AB_VARIANTS:-libcovt_base.so libcovt.so libcovt_base.so libcovt.so}; do
            echo "== $v"; COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/asm_run.py 20 2>&1 | grep -v amdgpu.ids || fatal asm_props_ab $?
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/props_run.py 2>&1 | grep -v amdgpu.ids || fatal asm_props_ab $?
        done ;;
    mvt_gpu) step mvt_gpu 300 python tools/mvt_vs_covt.py --gpu 9000 ;;
    fpfsize) step fpfsize 300 python -c "import sys; sys.path.insert(0, 'tools'); import op_breakdown; op_breakdown.fpf_scaling()" ;;
    prof) step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu ;;
    pmc_fetch) step rocprof_pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-props --no-assemble --no-strong-shards ;;
    pmc_write) step rocprof_pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-props --no-assemble --no-strong-shards ;;
    sq_fpf) step sq_fpf 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/sq_fpf -o run --output-format csv -- python tools/family_run.py fastpfor 2 ;;
    sq_fpf2) step sq_fpf2 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/sq_fpf2 -o run --output-format csv -- python tools/family_run.py fastpfor 2 ;;
    util_rle_props) OPB_PROPS=1 step $s 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/$s -o run --output-format csv -- python tools/family_run.py rle 2 ;;
    util_rle|util_varint|util_fastpfor|util_lane|util_all) fam=${s#util_}; step $s$sfx 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/$s$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 ;;
    sqi_rle|sqi_varint|sqi_fastpfor|sqi_lane|sqi_all) fam=${s#sqi_}; step $s$sfx 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/$s$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 ;;
    sqc_rle|sqc_varint|sqc_fastpfor|sqc_lane|sqc_all) fam=${s#sqc_}; step $s$sfx 600 rocprofv3 --pmc SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d gpurun_out/$s$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 ;;
    icache_rle|icache_varint|icache_fastpfor|icache_lane|icache_all) fam=${s#icache_}; step $s$sfx 600 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE -d gpurun_out/$s$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 ;;
    mem_rle|mem_varint|mem_fastpfor|mem_lane) fam=${s#mem_}; step $s$sfx 600 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d gpurun_out/$s$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 ;;
    sq_rle|sq_varint|sq_fastpfor|sq_lane) fam=${s#sq_}; step $s$sfx 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/$s$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 ;;
    opinst) step opinst 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/opinst -o run --output-format csv -- python tools/op_counters.py ;;
    tests_changed) step pytest_changed 600 python -u -m pytest tests/test_gpu_assembly.py tests/test_gpu_props.py tests/test_gpu_split.py tests/test_gpu_rle_adversarial.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    tests_r05) step pytest_r05 600 python -u -m pytest tests/test_gpu_assembly.py tests/test_gpu_props.py tests/test_jni_shim.py tests/test_gpu_device_plan.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -s ;;
    dplan_geo) step dplan_geo 200 python tools/device_plan_prof.py 20 --sweep --geometry ;;
    dplan_drop) step dplan_drop 300 python tools/device_plan_prof.py 20 --drop=16,64,256,1024,4096 ;;
    walk_timeline) step walk_timeline 300 python tools/walk_timeline.py 5 ;;
    dplan_prof_props) step dplan_prof_props 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dplan_prof_props -o run --output-format csv -- python tools/device_plan_prof.py 5 --props ;;
    dplan_sweep) step dplan_sweep 300 python tools/device_plan_prof.py 10 --sweep ;;
    dplan_props_sweep) step dplan_props_sweep 300 python tools/device_plan_prof.py 10 --sweep --props ;;
    dplan_ab) step dplan_ab 300 python tools/device_plan_ab.py 0 1 ;;
    dplan_var) for v in ${AB_VARIANTS:-libcovt.so}; do
            COVT_LIB_VARIANT=$v timeout -k 10 200 python tools/device_plan_prof.py 20 --sweep 2>&1 | grep -v amdgpu.ids || fatal dplan_var $?
        done ;;
    dplan_props_var) for v in ${AB_VARIANTS:-libcovt.so}; do
            COVT_LIB_VARIANT=$v timeout -k 10 200 python tools/device_plan_prof.py 20 --sweep --props 2>&1 | grep -v amdgpu.ids || fatal dplan_props_var $?
        done ;;
    dplan_prof_small) step dplan_prof_small 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dplan_prof_small -o run --output-format csv -- python tools/device_plan_prof.py 5 --small ;;
    dplan_props_small) step dplan_props_small 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dplan_props_small -o run --output-format csv -- python tools/device_plan_prof.py 5 --small --props ;;
    dplan_sq1) step dplan_sq1 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/dplan_sq1 -o run --output-format csv -- python tools/device_plan_prof.py 2 --props ;;
    dplan_sq2) step dplan_sq2 300 rocprofv3 --pmc SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d gpurun_out/dplan_sq2 -o run --output-format csv -- python tools/device_plan_prof.py 2 --props ;;
    dplan_api) step dplan_api 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/dplan_api -o run --output-format csv -- python tools/device_plan_prof.py 5 ;;
    dplan_prof_256) step dplan_prof_256 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dplan_prof_256 -o run --output-format csv -- python tools/device_plan_prof.py 5 --n256 ;;
    dplan_api_small) step dplan_api_small 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/dplan_api_small -o run --output-format csv -- python tools/device_plan_prof.py 20 --small --nosplit ;;
    dplan_sq_small) step dplan_sq_small 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d gpurun_out/dplan_sq_small -o run --output-format csv -- python tools/device_plan_prof.py 3 --small --nosplit ;;
    dplan_sorted) step dplan_sorted 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dplan_sorted -o run --output-format csv -- python tools/device_plan_prof.py 10 --sorted ;;
    timeline_shard8) step timeline_shard8 300 python tools/stream_timeline.py --shard=8/0 ;;
    shards_ratio) step shards_ratio 600 python tools/shard_sizes.py 20 --ns=4,8 --opts= \
            --opts=split_max_streams=0,split_ratio=200 --opts=split_max_streams=0,split_ratio=500 \
            --opts=split_max_streams=0,split_ratio=1000 --opts=split_max_streams=0,split_ratio=500,split_chunk=8192,split_values=8192 ;;
    shards_big) step shards_big 600 python tools/shard_sizes.py 20 --ns=1,4,8 --opts= \
            --opts=split_max_streams=0,split_ratio=1500,split_chunk=8192,split_values=8192 \
            --opts=split_max_streams=0,split_ratio=1500,split_chunk=16384,split_values=16384 \
            --opts=split_max_streams=0,split_ratio=2500,split_chunk=8192,split_values=8192 \
            --opts=split_max_streams=0,split_ratio=2500,split_chunk=4096,split_values=4096 ;;
    timeline_shard8s) step timeline_shard8s 300 python tools/stream_timeline.py --shard=8/0 --opts=split_max_streams=0 && \
        step timeline_shard4s 300 python tools/stream_timeline.py --shard=4/0 --opts=split_max_streams=0,split_ratio=2500,split_chunk=8192,split_values=8192 && \
        step timeline_shard4 300 python tools/stream_timeline.py --shard=4/0 ;;
    shards_layout) for v in ${AB_VARIANTS:-libcovt.so libcovt_sl1.so libcovt_sl2.so libcovt_sl3.so}; do
            echo "== layout $v"; COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/shard_sizes.py 20 --ns=4,8 \
            --opts=split_max_streams=0 --opts=split_max_streams=0,split_ratio=2500,split_chunk=8192,split_values=8192 \
            --opts=split_max_streams=0,split_ratio=6000,split_chunk=4096,split_values=4096 2>&1 | grep -A4 "slowest shard ms per N" || fatal shards_layout $?
        done ;;
    long_poles) step long_poles4 300 python tools/long_poles.py 20 --shard=4/0 && step long_poles8 300 python tools/long_poles.py 20 --shard=8/0 ;;
    shards_prio) for v in ${AB_VARIANTS:-libcovt.so libcovt_p0.so libcovt_L64.so libcovt_p3L64.so}; do
            echo "== prio $v"; COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/shard_sizes.py 20 --ns=1,4,8 --opts= --opts= 2>&1 | grep -A3 "slowest shard ms per N" || fatal shards_prio $?
        done ;;
    shards_cprio) for v in ${AB_VARIANTS:-libcovt.so libcovt_cp0.so libcovt_sl1.so}; do
            echo "== chunk prio $v"; COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/shard_sizes.py 20 --ns=1,4,8,16 --opts= --opts=split_max_streams=0 \
            --opts=split_max_streams=0,split_chunk=8192,split_values=8192 --opts=split_max_streams=0,split_ratio=2000,split_chunk=8192,split_values=8192 2>&1 | grep -A5 "slowest shard ms per N" || fatal shards_cprio $?
        done ;;
    shards_chunk) step shards_chunk 900 python tools/shard_sizes.py 20 --ns=8,16,32,64 --configs --opts= --opts=split_max_streams=0 \
            --opts=split_max_streams=0,split_chunk=4096,split_values=4096 --opts=split_max_streams=0,split_chunk=8192,split_values=8192 \
            --opts=split_max_streams=0,split_chunk=16384,split_values=16384 ;;
    shards_grow) step shards_grow 900 python tools/shard_sizes.py 20 --ns=1,2,4,8,16,32,64 --configs --opts= --opts=split_grow=0,split_max_streams=32768 ;;
    n4) step timeline_n4s 300 python tools/stream_timeline.py --shard=4/0 --opts=split_max_streams=0 && \
        step shards_n4 600 python tools/shard_sizes.py 20 --ns=4,8 --opts= --opts=split_max_streams=0 --opts=split_max_streams=0,fpf_split_weight=2 \
            --opts=split_max_streams=0,split_ratio=6000 --opts=split_max_streams=0,split_ratio=1500 ;;
    shards_w) for v in ${AB_VARIANTS:-libcovt.so libcovt_sl1.so}; do
            echo "== $v"; COVT_LIB_VARIANT=$v timeout -k 10 400 python tools/shard_sizes.py 20 --ns=2,4,8,16,32 --configs --opts= --opts=split_max_streams=0 \
            --opts=fpf_split_weight=2 --opts=split_max_streams=0,fpf_split_weight=2 2>&1 | grep -A5 "slowest shard ms per N" || fatal shards_w $?
        done ;;
    fetch_fpf_ab) for v in ${AB_VARIANTS:-libcovt_prev.so libcovt.so libcovt_s8.so}; do
            COVT_LIB_VARIANT=$v step fetch_fpf_$v 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fetch_fpf_$v -o run --output-format csv -- python tools/family_run.py fastpfor 2
        done ;;
    dplan_lib) rm -f gpurun_out/dplan_lib.log; for v in ${AB_VARIANTS:-libcovt_r0.so libcovt.so libcovt_r0.so libcovt.so}; do
            echo "== $v" >> gpurun_out/dplan_lib.log
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/device_plan_prof.py 20 >> gpurun_out/dplan_lib.log 2>&1 || fatal dplan_lib $?
        done ;;
    tests_dplan) step pytest_dplan 600 python -u -m pytest tests/test_gpu_device_plan.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    tests_fpf) step pytest_fpf 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    deep_shards) rm -f gpurun_out/deep_shards.log; for v in ${AB_VARIANTS:-libcovt_d0.so libcovt.so libcovt_deep6.so}; do
            echo "== $v" >> gpurun_out/deep_shards.log
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/shard_sizes.py 20 --ns=4,8,16 --opts= --opts= >> gpurun_out/deep_shards.log 2>&1 || fatal deep_shards $?
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/long_poles.py 20 --shard=8/0 >> gpurun_out/deep_shards.log 2>&1 || fatal deep_shards $?
        done ;;
    shards_n4r) step shards_n4r 600 python tools/shard_sizes.py 20 --ns=2,4,8 --opts= --opts=split_max_streams=0 --opts=split_max_streams=0,split_ratio=6000 \
            --opts=split_max_streams=0,split_ratio=12000 --opts=split_ratio=6000 ;;
    sq_rle_abl) for v in libcovt.so libcovt_abl_ABL_RLE_NOLIT.so libcovt_abl_ABL_RLE_NORUN.so; do
            OPB_PROPS=1 COVT_LIB_VARIANT=$v step sq_rle_abl_$v 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/sq_rle_abl_$v -o run --output-format csv -- python tools/family_run.py rle 2
        done ;;
    sq_dplan) step sq_dplan 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/sq_dplan -o run --output-format csv -- python tools/device_plan_prof.py 3 ;;
    sq_dplan_props) step sq_dplan_props 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/sq_dplan_props -o run --output-format csv -- python tools/device_plan_prof.py 3 --props ;;
    dplan_lib_props) rm -f gpurun_out/dplan_lib_props.log; for v in ${AB_VARIANTS:-libcovt_dp0.so libcovt.so libcovt_dp0.so libcovt.so}; do
            echo "== $v" >> gpurun_out/dplan_lib_props.log
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/device_plan_prof.py 10 --props >> gpurun_out/dplan_lib_props.log 2>&1 || fatal dplan_lib_props $?
        done ;;
    sq_asm_passes) for v in libcovt_asm1.so libcovt_asm2.so libcovt.so; do
            COVT_LIB_VARIANT=$v step sqa_$v 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/sqa_$v -o run --output-format csv -- python tools/asm_run.py 2 && \
            COVT_LIB_VARIANT=$v step mema_$v 300 rocprofv3 --pmc TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d gpurun_out/mema_$v -o run --output-format csv -- python tools/asm_run.py 2
        done ;;
    sq_dplan_var) for v in ${AB_VARIANTS:-libcovt.so libcovt_pl2.so}; do
            COVT_LIB_VARIANT=$v step sqd_$v 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/sqd_$v -o run --output-format csv -- python tools/device_plan_prof.py 2
        done ;;
    shards_n4b) step shards_n4b 600 python tools/shard_sizes.py 20 --ns=4 --opts= --opts=split_max_streams=0,split_ratio=1600 \
            --opts=split_max_streams=0,split_ratio=1800 --opts=split_max_streams=0,split_ratio=2000 --opts=split_max_streams=0,split_ratio=2400 ;;
    shards) step shard_sizes 300 python tools/shard_sizes.py 30 ;;
    shards_policy) step shards_policy 600 python tools/shard_sizes.py 20 --ns=1,2,4,8,16 --opts= \
            --opts=lane_min_streams=16384,split_max_streams=0 --opts=split_max_streams=16384 --opts=split_max_streams=0 ;;
    ops_props) OPB_PROPS=1 step ops_props 600 python tools/op_breakdown.py ;;
    props_time) step props_time 300 python tools/props_run.py ;;
    fetch_fastpfor|fetch_varint|fetch_rle|fetch_lane|fetch_rle_props|fetch_lane_props) fam=${s#fetch_}; fam=${fam%_props}
        if [ "${s%_props}" != "$s" ]; then export OPB_PROPS=1; else unset OPB_PROPS; fi
        step $s$sfx 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$s$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 ;;
    sq_rle_props) OPB_PROPS=1 step $s 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVES -d gpurun_out/$s -o run --output-format csv -- python tools/family_run.py rle 2 ;;
    config1_prof) step config1_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/config1_prof -o run --output-format csv -- python tools/config1_prof.py 20 ;;
    config1_passes) for v in libcovt_asm1.so libcovt_asm2.so libcovt_asm3.so libcovt.so; do
            COVT_LIB_VARIANT=$v step config1_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/config1_$v -o run --output-format csv -- python tools/config1_prof.py 20
        done ;;
    dplan_props) step dplan_props 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dplan_props -o run --output-format csv -- python tools/device_plan_prof.py 5 --props ;;
    launch_modes) step launch_modes 300 python tools/launch_mode_ab.py ;;
    dplan_prof) step dplan_prof 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/dplan_prof -o run --output-format csv -- python tools/device_plan_prof.py 10 ;;
    sqi_fpf_var) for v in ${AB_VARIANTS:-libcovt_base.so libcovt.so}; do
            COVT_LIB_VARIANT=$v step sqi_fpf_$v 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/sqi_fpf_$v -o run --output-format csv -- python tools/family_run.py fastpfor 2 && \
            COVT_LIB_VARIANT=$v step sqw_fpf_$v 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU -d gpurun_out/sqw_fpf_$v -o run --output-format csv -- python tools/family_run.py fastpfor 2 || exit $?
        done ;;
    fpf_probe) for v in ${AB_VARIANTS:-libcovt_base.so libcovt.so libcovt_base.so libcovt.so}; do
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/fpf_probe.py 20 2>&1 | grep -v amdgpu.ids || fatal fpf_probe $?
        done ;;
    timeline_ab) step timeline_old 300 env TIMING_LIB=libcovt_timing_old.so python tools/stream_timeline.py && \
        step timeline_new 300 python tools/stream_timeline.py ;;
    abprops) step ab_props 900 env AB_PROPS=1 python tools/ab.py ${AB_VARIANTS:-libcovt_base.so libcovt.so} ;;
    sq_families) for fam in fastpfor varint rle lane; do  # -> tools/pmc_families.py
            step sqi_$fam$sfx 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/sqi_$fam$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 && \
            step sqw_$fam$sfx 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d gpurun_out/sqw_$fam$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 || exit $?
        done
        python tools/pmc_families.py gpurun_out $sfx > gpurun_out/pmc_families$sfx.txt ;;
    tcc_families) for fam in fastpfor varint rle lane; do
            step tcc_$fam$sfx 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d gpurun_out/tcc_$fam$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 && \
            step fetch_$fam$sfx 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fetch_$fam$sfx -o run --output-format csv -- python tools/family_run.py $fam 2 || exit $?
        done ;;
    shards_ab) for v in ${AB_VARIANTS:-libcovt_r5.so libcovt.so libcovt_r5.so libcovt.so}; do
            echo "== $v" >> gpurun_out/shards_ab.log
            COVT_LIB_VARIANT=$v timeout -k 10 300 python tools/shard_sizes.py 15 --ns=${SHARD_NS:-1,2,4,8} >> gpurun_out/shards_ab.log 2>&1 || fatal shards_ab $?
        done ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "session done"
