#!/bin/bash
# One profiling session on the gpurun box for profiles/<round>/: kernel trace + stats of the bench
# launch alone (no property / assembly / config / PCIe legs, so the per-kernel rows describe only the
# config-5 decode launch), launch spans, FETCH_SIZE and WRITE_SIZE in separate --pmc passes (->
# profiles/pmc_traffic.json, which the bench line's roofline.traffic reads), then the full bench line.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${1:-r03}
mkdir -p gpurun_out "gpurun_out/$R"
LEAN="--no-cpu --no-props --no-assemble --no-configs --no-strong-shards --e2e-reps 0 --abi-host-reps 0 --device-plan-reps 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 $LEAN > "gpurun_out/$R/prof_bench.json" 2> "gpurun_out/$R/prof_bench.err"
python tools/launch_span.py gpurun_out/prof/run_kernel_trace.csv > "gpurun_out/$R/rocprof_launch_spans.txt"
cp gpurun_out/prof/run_kernel_stats.csv "gpurun_out/$R/rocprof_kernel_stats.csv"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 $LEAN > /dev/null 2> "gpurun_out/$R/pmc_fetch.err"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 $LEAN > /dev/null 2> "gpurun_out/$R/pmc_write.err"
python tools/pmc_traffic.py gpurun_out > "gpurun_out/$R/pmc_traffic.txt"
cp profiles/pmc_traffic.json "gpurun_out/$R/pmc_traffic.json"
timeout -k 10 600 python bench.py > "gpurun_out/$R/bench.json" 2> "gpurun_out/$R/bench.err"
timeout -k 10 300 python tools/config_timeline.py > "gpurun_out/$R/config_timeline.txt" 2>&1
timeout -k 10 300 python tools/op_breakdown.py > "gpurun_out/$R/op_breakdown.txt" 2>&1
OPB_PROPS=1 timeout -k 10 300 python tools/op_breakdown.py > "gpurun_out/$R/op_breakdown_props.txt" 2>&1
echo "profile session done"
