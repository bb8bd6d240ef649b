#!/bin/bash
# Build libcovt_base.so from HEAD (the working tree's changes stashed meanwhile) for A/B runs.
set -e
cd "$(dirname "$0")/.."
git stash -q
make -s -C cov-tiles_amd libcovt.so && cp cov-tiles_amd/libcovt.so cov-tiles_amd/libcovt_base.so
git stash pop -q
make -s -C cov-tiles_amd libcovt.so timing
