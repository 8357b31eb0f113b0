#!/bin/bash
# Host-side ASan + UBSan build of the kernel library's launch planners (tools/host_sanitize.cpp)
# and a CPU run of the planner sweep.  -fsanitize=... applies to host code only (-Xarch_host);
# the gfx950 device code is compiled normally (GPU sanitizers are not available on this pool).
set -eo pipefail
cd "$(dirname "$0")/.."
out=${OUT:-build/host_sanitize}
mkdir -p "$out"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer"
objs=()
for f in csrc/conv3x3_res.hip csrc/conv3x3_fwd.hip csrc/conv3x3_wgrad.hip csrc/bn.hip csrc/reduce.hip csrc/head_ce.hip csrc/misc.hip csrc/convt_gemm.hip; do
  o="$out/$(basename "$f" .hip).o"
  hipcc --offload-arch=gfx950 -std=c++17 -O1 -g $SAN -Icsrc -c "$f" -o "$o" &
  objs+=("$o")
done
wait
hipcc --offload-arch=gfx950 -std=c++17 -O1 -g $SAN -Icsrc -x hip -c tools/host_sanitize.cpp -o "$out/host_sanitize.o"
hipcc --offload-arch=gfx950 $SAN "$out/host_sanitize.o" "${objs[@]}" -o "$out/host_sanitize"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$out/host_sanitize"
