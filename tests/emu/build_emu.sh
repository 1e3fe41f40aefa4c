#!/bin/bash
# TEST INFRASTRUCTURE: build libkueue_tas_emu.so — the unmodified product
# sources (kernels + device layer + host layer) compiled with g++ against the
# CPU SIMT emulator in tests/emu/hip/hip_runtime.h.  Output: tests/emu/_build/.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(cd "$HERE/../.." && pwd)"
OUT="$HERE/_build"
mkdir -p "$OUT/src"
CSRC="$ROOT/kueue_oss_amd/csrc"
# dynamic LDS: `extern __shared__ T name[];` has no static-local equivalent
# - dynamic LDS: `extern __shared__ T name[];` has no static-local equivalent
# - lockstep: on hardware the 64 lanes of a wave execute the (wave-uniform)
#   counter stores of phase 2 in lockstep; fibers do not, so every store of a
#   domain counter becomes a wave-synchronization point here.
# - per-wave state: select_kernel keeps the wave's descriptor / result header /
#   out-parameters in LDS, stored alike by all (lockstep) lanes; fibers are
#   not lockstep, so each lane keeps a private copy instead.
sed -e 's/extern __shared__ Key lds_all\[\];/Key* lds_all = static_cast<Key*>(emu::dynamic_lds());/' \
    -e 's/extern __shared__ uint32_t touched_lds\[\];/uint32_t* touched_lds = static_cast<uint32_t*>(emu::dynamic_lds());/' \
    -e 's/^  __shared__ \(Wave sh_wave\|kueue_tas_eval_out sh_out\|int sh_ints\)/  \1/' \
    -e 's/^    own(g);$/    emu::wave_barrier(); own(g);/' \
    -e 's/^    ov\[int64_t(f) \* SD + g\] = v;/    ov[int64_t(f) * SD + g] = v; emu::wave_barrier();/' \
  "$CSRC/tas_kernels.hip" > "$OUT/src/tas_kernels.hip"
grep -q 'emu::wave_barrier(); own(g);' "$OUT/src/tas_kernels.hip" || { echo "lockstep patch failed"; exit 1; }
grep -q '= v; emu::wave_barrier();' "$OUT/src/tas_kernels.hip" || { echo "lockstep patch failed"; exit 1; }
grep -q '^  Wave sh_wave\[' "$OUT/src/tas_kernels.hip" || { echo "per-wave state patch failed"; exit 1; }
grep -q '^  __shared__ \(Wave\|kueue_tas_eval_out\|int sh_ints\)' "$OUT/src/tas_kernels.hip" && { echo "per-wave state patch incomplete"; exit 1; }
cp "$CSRC/tas_internal.h" "$CSRC/json_reader.h" "$CSRC/label_selectors.h" "$CSRC/tas_balanced.h" \
   "$CSRC/tas_pool.h" "$OUT/src/"
sed "s#\"../../include/#\"#" "$CSRC/tas_internal.h" > "$OUT/src/tas_internal.h"
cp "$ROOT/include/kueue_tas.h" "$ROOT/include/kueue_tas_debug.h" "$OUT/src/"
cp "$CSRC/tas_device.hip" "$OUT/src/tas_device.cpp"
sed "s#\"../../include/#\"#" "$CSRC/tas_host.cpp" > "$OUT/src/tas_host.cpp"
CXXFLAGS="${CXXFLAGS:--O1 -g}"
g++ -std=c++17 $CXXFLAGS -ffp-contract=off -fPIC -shared -pthread -I"$HERE" -I"$OUT/src" \
  "$OUT/src/tas_device.cpp" "$OUT/src/tas_host.cpp" "$HERE/hip_emu.cpp" -o "$OUT/libkueue_tas_emu.so"
echo "$OUT/libkueue_tas_emu.so"
