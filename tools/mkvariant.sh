#!/bin/bash
# Build cov-tiles_amd/libcovt_NAME.so for paired A/B runs: one translation unit of the working tree
# compiled with extra flags (e.g. -DCOVT_FW_SPAN=256), linked with the other objects of libcovt.so.
#   tools/mkvariant.sh NAME UNIT FLAGS...     UNIT: covt_decode | covt_plan_device | covt_host | ...
set -e
cd "$(dirname "$0")/.."
NAME=$1; UNIT=$2; shift 2
make -s -C cov-tiles_amd libcovt.so
mkdir -p /tmp/covt_var
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics"
SRC=cov-tiles_amd/csrc/$UNIT.hip; [ -f "$SRC" ] || SRC=cov-tiles_amd/csrc/$UNIT.cpp
$H -Iinclude -Icov-tiles_amd/csrc "$@" -c -o /tmp/covt_var/$NAME.o "$SRC"
OBJS=""
for u in covt_decode covt_assemble covt_props covt_plan_device covt_host; do
    if [ "$u" = "$UNIT" ]; then OBJS="$OBJS /tmp/covt_var/$NAME.o"; else OBJS="$OBJS cov-tiles_amd/csrc/$u.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o cov-tiles_amd/libcovt_$NAME.so $OBJS -lpthread
echo "libcovt_$NAME.so: $UNIT with $*"
