#!/bin/bash
# A/B of variant libraries built into smallpt-enoki-optix_amd/build_<name>/:
# VARLIBS="base cam" CONFIGS="1 4" ROUNDS=2 tools/ab_variants.sh  (X=0: build/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/smallpt-enoki-optix_amd
V="X=0"
for n in ${VARLIBS:-}; do V="$V SPT_LIB=$L/build_$n/libspt.so"; done
CONFIGS="${CONFIGS:-1}" ROUNDS="${ROUNDS:-2}" VARIANTS="$V" bash tools/ov.sh
