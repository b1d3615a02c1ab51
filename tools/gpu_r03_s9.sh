#!/bin/bash
# Round-3 call 9: same-box A/B of the spill-free eval_tile5 (buffer-load DMA and
# room rows, per-tile lane offsets); GPU suite; bench with live PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s9}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step ab_med 240 python -u tools/ab_eval.py med 65536 base3:8 nospill:8
step ab_lg 240 python -u tools/ab_eval.py lg 65536 base3:8 nospill:8
step ab_comp 240 python -u tools/ab_eval.py comp01 65536 base3:8 nospill:8
bash tools/gpu_check.sh $T tests bench prof || exit $?
echo done
