#!/bin/bash
# Round-3 call 7: same-box A/B of the Move1 window variants and the matcher's
# writelane transpose / ballot builtin.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s7}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 700 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step abls_comp01 300 python -u tools/ab_ls.py comp01 8192 base2 win win2 bw
step abls_med 300 python -u tools/ab_ls.py med 4096 base2 win win2 bw
step abls_lg 300 python -u tools/ab_ls.py lg 4096 base2 win2 bw
step ab_med 240 python -u tools/ab_eval.py med 65536 base2:8 bw:8
echo done
