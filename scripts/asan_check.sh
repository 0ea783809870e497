#!/bin/bash
# Host-side AddressSanitizer run of the C ABI (no GPU needed).
# Builds libpetdiff.so with ASan on its HOST code (hipcc: -Xarch_host -fsanitize=address; device code
# is unchanged, GPU sanitizers are not available on this pool) and the MH C checker with clang ASan,
# then runs the CPU suites that exercise them through ctypes: tests/test_abi.py (symbol table,
# config, schedule restatement, every error path of petdiff_create) and tests/test_cpu_mh.py (the C
# MH sampler against the NumPy restatement).  Output: build/asan/ (git-ignored).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/asan"
LLVM=/opt/rocm/lib/llvm
RT="$(ls "$LLVM"/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n1)"
JOBS="${MAX_JOBS:-8}"
mkdir -p "$OUT"
make -C "$ROOT/pet_posterior_distribution_amd/csrc" -j"$JOBS" OUT="$OUT/libpetdiff.so" OBJDIR="$OUT/obj" \
  EXTRA="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -g" \
  LDEXTRA="-fsanitize=address -fno-gpu-sanitize -shared-libasan"
"$LLVM/bin/clang" -O1 -g -fno-omit-frame-pointer -fsanitize=address -shared-libasan -fopenmp -fPIC -std=c11 \
  -shared "$ROOT/oracle/mh_ref.c" -o "$OUT/libmhref.so" -lm
cd "$ROOT"
LD_PRELOAD="$RT" ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1" \
  PETDIFF_LIB="$OUT/libpetdiff.so" MHREF_LIB="$OUT/libmhref.so" \
  python -m pytest tests/test_abi.py tests/test_cpu_mh.py -q -p no:cacheprovider "$@"
