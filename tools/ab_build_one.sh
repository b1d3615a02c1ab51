#!/bin/bash
# Same-box A/B build of ONE source file of the working tree with extra flags
# (HIPX), linked with the in-tree objects of the others (make first):
#   HIPX=-DTT_T5_PRIO=1 tools/ab_build_one.sh tt_eval prio
set -eu
REPO=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; NAME=$2
PKG="$REPO/timetabling-ga-mpi-openmp_amd"
TMP=$(mktemp -d /tmp/ab1_XXXX)
mkdir -p "$REPO/ab_libs"
(cd "$PKG" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC ${HIPX:-} -c "csrc/$SRC.hip" -o "$TMP/$SRC.o")
objs="$TMP/$SRC.o"
for o in "$PKG"/build/*.o; do [ "$(basename "$o" .o)" = "$SRC" ] || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$REPO/ab_libs/libttga_$NAME.so" $objs
rm -rf "$TMP"
echo "$REPO/ab_libs/libttga_$NAME.so"
