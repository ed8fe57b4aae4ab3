#!/bin/bash
# Build a variant of lib/libqsmd.so into ablib/NAME.so (diagnostic / A-B
# builds; ablib/ is git-ignored but travels to the GPU box), from a copy of
# the sources with the given patches applied and extra compiler flags:
#   tools/build_variant.sh NAME "FLAGS" [PATCH ...]
# e.g. the stage-0 diagnostic builds (tools/diag/compact_diag.patch: without
# the search, per-group phase stamps for tools/stage0_anatomy.py, no
# heavy-list append):
#   tools/build_variant.sh nosearch "-DQSMD_DIAG_STAGE0=1" tools/diag/compact_diag.patch
#   tools/build_variant.sh stamps   "-DQSMD_DIAG_STAGE0=2" tools/diag/compact_diag.patch
#   tools/build_variant.sh noheavy  "-DQSMD_DIAG_NOHEAVY=1" tools/diag/compact_diag.patch
set -e
NAME=$1; FLAGS=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/quickcheck-state-machine-distributed_amd
OUT=$ROOT/ablib/$NAME
SRC=$OUT/csrc
rm -rf "$SRC" && mkdir -p "$SRC"
cp "$PKG"/csrc/*.hip "$PKG"/csrc/*.h "$SRC"/
for p in "$@"; do
  patch -s -d "$SRC" -p0 < "$ROOT/$p"
done
objs=()
for f in compact memo wave gen wellformed split api; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -I"$ROOT/include" -I"$SRC" $FLAGS \
    -c "$SRC/$f.hip" -o "$OUT/$f.o" &
  objs+=("$OUT/$f.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$ROOT/ablib/$NAME.so"
echo "ablib/$NAME.so"
