#!/bin/bash
# Build and run csrc/tests/host_checks.cpp with AddressSanitizer + UndefinedBehaviorSanitizer on
# the HOST code only (GPU sanitizers are not available on this pool; -fsanitize flags go behind
# -Xarch_host). CPU only: no GPU is touched.
set -euo pipefail
cd "$(dirname "$0")/.."
out=${TMPDIR:-/tmp}/cs336_host_checks
hipcc -O1 -g -std=c++17 --offload-arch=gfx950 -x hip \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all \
  -Icsrc/include -Icsrc/flash_attn csrc/tests/host_checks.cpp -o "$out"
ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1 "$out"
