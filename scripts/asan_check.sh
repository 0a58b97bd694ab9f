#!/bin/bash
# Host sanitizer run ("ASan/UBSan on the CPU restatement"), CPU only, no GPU.
#
# Builds the host-instrumented libmeshsearch (mesh_amd/csrc `make asan`: C ABI, blob header parser, device plan,
# OBJ/PLY loaders; the gfx950 code objects are not instrumented) and the instrumented oracle (oracle `make asan`),
# both with the HIP toolchain's clang so one ASan runtime serves the process, then runs with that runtime
# preloaded:
#   * the non-GPU tests of the loaders, the ABI / header / validation surface and the oracle against the reference's
#     golden vectors (tests/test_loaders.py, tests/test_abi.py, tests/test_oracle.py);
#     (less test_build_id_matches_sources -- the sanitized build has its own id -- and the bound-check test, run below);
#   * tests/csrc/bound_check.cpp (the kernels' fp32 bound code on the host) built with the same sanitizers.
# Leak checking is off (the Python interpreter keeps its allocations); any ASan report or UBSan error aborts.
#
#     bash scripts/asan_check.sh [log]      (default log: profiles/r06_asan_check.log)
set -u
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r06_asan_check.log}
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
{
  echo "# asan_check.sh at $(git rev-parse --short HEAD) ($(date -u +%Y-%m-%dT%H:%MZ)), runtime $RT"
  make -s -j8 -C mesh_amd/csrc asan && make -s -C oracle asan || { echo "BUILD FAILED"; exit 2; }
  echo "## pytest (loaders, ABI, oracle) with the sanitized libraries"
  LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    MESH_AMD_LIB=$PWD/build/asan/libmeshsearch.so ORACLE_LIB=$PWD/oracle/_build/asan/liboracle.so \
    MESH_AMD_ASAN_CHECK=1 \
    python -m pytest tests/test_loaders.py tests/test_abi.py tests/test_oracle.py -q -m "not gpu" -p no:cacheprovider \
      -k "not child_box_bound and not build_id_matches_sources" 2>&1
  rc1=$?
  echo "pytest rc=$rc1"
  echo "## bound_check (host build of the kernels' bound code) under ASan + UBSan"
  exe=build/asan/bound_check
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -ffp-contract=off --offload-arch=gfx950 -x hip tests/csrc/bound_check.cpp \
    -I mesh_amd/csrc -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
    -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer -o $exe 2>&1 &&
    ASAN_OPTIONS=abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 $exe 100000 2>&1 | tail -3
  rc2=${PIPESTATUS[0]}
  echo "bound_check rc=$rc2"
  echo "## result: pytest rc=$rc1 bound_check rc=$rc2"
} > "$LOG" 2>&1
tail -4 "$LOG"
