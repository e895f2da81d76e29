#!/bin/bash
# Build a variant of the package into variants/<name>/ (same sources, extra -D
# flags) for same-box A/B timing: TSA_PKG_DIR=variants/<name> selects it.
# The diagnostic knobs (TSA_LAP_SINGLE, TSA_LAP_RING_SLACK, TSA_LAP_FULL_RINGS,
# per-phase cycle counters) exist only in a -DTSA_DIAG build:
#   scripts/build_variant.sh diag "-DTSA_DIAG"
#   scripts/build_variant.sh nopf "-DTSA_A_PREFETCH=0"
set -e
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2
PKG=hw-accelerator-three-sequence-alignment_amd
SRC=${SRC:-$PKG}  # source tree (e.g. a git archive of an older commit)
OUT=variants/$NAME
rm -rf "$OUT"; mkdir -p "$OUT/lib" "$OUT/build"
cp $PKG/*.py "$OUT/"
# ONLY="pencil_kernel lap_kernel": recompile just those sources with DEFS and
# take the others' objects from the main build ($PKG/build, `make` first) --
# a knob that touches one kernel file then costs one compile, not five
objs=()
for f in $SRC/csrc/*.hip; do
  b=$(basename "${f%.hip}")
  o="$OUT/build/$b.o"
  if [ -n "$ONLY" ] && ! echo " $ONLY " | grep -q " $b "; then
    cp "$PKG/build/$b.o" "$o"
  else
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function \
      -DTSA_SRC_HASH="\"variant-$NAME\"" $DEFS -c "$f" -o "$o" &
  fi
  objs+=("$o")
done
wait
for o in "${objs[@]}"; do [ -f "$o" ] || { echo "build_variant: $o failed" >&2; exit 1; }; done
# the kernel resource table (tools/kernel_meta.py; a tree without it links it unused)
python3 $PKG/tools/kernel_meta.py --cpp "$OUT/build/kernel_meta.cpp" "${objs[@]}" > /dev/null
g++ -O2 -std=c++17 -fPIC -I$PKG/csrc -c "$OUT/build/kernel_meta.cpp" -o "$OUT/build/kernel_meta.o"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared -o "$OUT/lib/libtrialign.so" "${objs[@]}" \
  "$OUT/build/kernel_meta.o" -lpthread
rm -rf "$OUT/build"
echo "built $OUT"
