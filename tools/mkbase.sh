#!/bin/bash
# Build cov-tiles_amd/libcovt_base.so for paired A/B runs: the decode kernels (csrc/covt_decode.hip) of
# git revision REV (default HEAD) linked with the working tree's host code and other kernels, so the two
# libraries differ only in the decode kernels and export the same C-ABI.
#   tools/mkbase.sh [REV]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
mkdir -p /tmp/covt_base
git show "$REV:cov-tiles_amd/csrc/covt_decode.hip" > /tmp/covt_base/covt_decode.hip
make -s -C cov-tiles_amd libcovt.so
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics"
$H -Iinclude -Icov-tiles_amd/csrc -c -o /tmp/covt_base/covt_decode.o /tmp/covt_base/covt_decode.hip
cd cov-tiles_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libcovt_base.so /tmp/covt_base/covt_decode.o \
    csrc/covt_assemble.o csrc/covt_props.o csrc/covt_plan_device.o csrc/covt_host.o -lpthread
echo "libcovt_base.so: decode kernels of $(git rev-parse --short "$REV")"
