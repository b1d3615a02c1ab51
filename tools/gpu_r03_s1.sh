#!/bin/bash
# Round-3 call: the GPU test suite, smoke, same-box A/B of the dword B rows, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s1}; O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_check.sh $T tests smoke || exit $?
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 800 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step ab_med 240 python -u tools/ab_eval.py med 65536 head:8 b32:8
step ab_lg 240 python -u tools/ab_eval.py lg 65536 head:8 b32:8
step ab_syn 300 python -u tools/ab_eval.py syn 262144 head:13 b32:13
bash tools/gpu_check.sh $T bench
