#!/bin/bash
# Build libttga.so from the csrc/ of a git revision (or the working tree: "wt")
# into ab_libs/libttga_<name>.so, for same-box A/B timing (tools/ab_eval.py).
# usage: tools/ab_build.sh <rev|wt> <name>
set -eu
REPO=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
SRC=$(mktemp -d /tmp/ab_XXXX)
mkdir -p "$SRC/x/csrc" "$SRC/include" "$REPO/ab_libs"
if [ "$REV" = wt ]; then
  cp "$REPO"/timetabling-ga-mpi-openmp_amd/csrc/* "$SRC/x/csrc/"; cp "$REPO"/include/ttga.h "$SRC/include/"
else
  git -C "$REPO" archive "$REV" timetabling-ga-mpi-openmp_amd/csrc include/ttga.h | tar -x -C "$SRC"
  mv "$SRC"/timetabling-ga-mpi-openmp_amd/csrc/* "$SRC/x/csrc/"
fi
mkdir -p "$SRC/obj"
for f in "$SRC"/x/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC ${HIPX:-} -c "$f" -o "$SRC/obj/$(basename "$f" .hip).o" &
  pids="${pids:-} $!"
done
for p in $pids; do wait $p || { echo "compile failed" >&2; rm -rf "$SRC"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$REPO/ab_libs/libttga_$NAME.so" "$SRC"/obj/*.o
rm -rf "$SRC"
echo "$REPO/ab_libs/libttga_$NAME.so"
