#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer build of everything that
# runs on the CPU (VERDICT r1 "do this" 7): the OBJ / pbrt-v3 / PLY readers,
# the host BVH2 and BVH8 builders, the C ABI's host code and the oracle, all
# with clang (one ASan runtime in the process; the device code is built as
# usual — sanitizers are host-only: -Xarch_host before each -fsanitize=).
# Then the CPU test files that drive those parsers and builders run against
# the sanitized libraries.  Log: profiles/sanitize_r02.log (committed).
#   usage: tools/sanitize.sh [LOG]
set -eu -o pipefail
cd "$(dirname "$0")/.."
log=${1:-profiles/sanitize_r02.log}
CLANG=/opt/rocm/lib/llvm/bin/clang
SAN="-g -O1 -fno-omit-frame-pointer -fno-sanitize-recover=all"
# hipcc sources: host side only (-Xarch_host); -x c++ sources: HOSTEXTRA
make -s -C smallpt-enoki-optix_amd BUILD=build_asan \
    EXTRA="$SAN -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined" \
    HOSTEXTRA="-fsanitize=address,undefined" build_asan/libspt.so
mkdir -p oracle/build_asan
$CLANG -std=c11 -fPIC -ffp-contract=off -pthread $SAN -fsanitize=address,undefined -shared \
    -o oracle/build_asan/liboracle.so oracle/oracle.c -lm
RT=$($CLANG -print-file-name=libclang_rt.asan-x86_64.so)
UBRT=$(dirname "$RT")/libclang_rt.ubsan_standalone-x86_64.so
{
  echo "# tools/sanitize.sh  $(date -u +%FT%TZ)  $(git rev-parse --short HEAD)"
  echo "# libspt.so (host code: ASan+UBSan) = smallpt-enoki-optix_amd/build_asan/libspt.so"
  echo "# oracle = oracle/build_asan/liboracle.so ; runtime = $RT"
  nm smallpt-enoki-optix_amd/build_asan/libspt.so | grep -c "__asan_report" | sed 's/^/# asan report sites in libspt.so: /'
  nm oracle/build_asan/liboracle.so | grep -c "__asan_report" | sed 's/^/# asan report sites in liboracle.so: /'
} > "$log"
env ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    LD_PRELOAD="$RT" SPT_LIB="$PWD/smallpt-enoki-optix_amd/build_asan/libspt.so" \
    ORACLE_LIB="$PWD/oracle/build_asan/liboracle.so" \
    python -m pytest tests/test_host.py tests/test_pbrt.py tests/test_oracle.py tests/test_sanitize_inputs.py \
        -q -p no:cacheprovider 2>&1 | tee -a "$log"
