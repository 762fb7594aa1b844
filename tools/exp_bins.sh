#!/bin/bash
# Host binned-SAH bin count: 32 (default) vs 64 vs 256 on config 1 (host-built BVH).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
VARIANTS="b32= b64=$P/build_b64/libspt.so b256=$P/build_b256/libspt.so" ROUNDS=3 timeout -k 10 500 bash tools/ab.sh || exit $?
