#!/bin/bash
# Build csrc/tests/host_selftest.cpp together with the kernel translation units
# (whose *_host twins it drives) and the store worker (StoreCore links its launcher;
# the self test runs StoreCore's host twin) with AddressSanitizer + UndefinedBehaviorSanitizer
# on the HOST side only, and run it.  Device code is compiled normally: GPU
# sanitizers are not used.  No GPU is needed to run it.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=build/sanitize
mkdir -p "$OUT"
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer
     -Xarch_host -fno-sanitize-recover=undefined)
FLAGS=(-x hip --offload-arch=gfx950 -O1 -g -std=c++17 -ffp-contract=off -Icsrc/include -I/opt/rocm/include)
SRCS=(csrc/hip/audit_kernels.hip csrc/hip/governance_kernels.hip csrc/hip/liability_kernels.hip
      csrc/hip/session_kernels.hip csrc/hip/saga_kernels.hip csrc/hip/pipeline.hip csrc/hip/store_worker.hip
      csrc/tests/host_selftest.cpp)
OBJS=()
pids=()
for s in "${SRCS[@]}"; do
  o="$OUT/$(basename "${s%.*}").o"
  OBJS+=("$o")
  # rebuild only what changed (the source, or any shared header, is newer than its object)
  if [[ -f "$o" && "$o" -nt "$s" && -z "$(find csrc/include -newer "$o" -name '*.h' -print -quit)" ]]; then continue; fi
  /opt/rocm/bin/hipcc "${FLAGS[@]}" "${SAN[@]}" -c "$s" -o "$o" &
  pids+=($!)
done
for p in "${pids[@]+"${pids[@]}"}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=address,undefined -fno-gpu-sanitize "${OBJS[@]}" -o "$OUT/host_selftest" \
  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 "$OUT/host_selftest"
