#!/bin/bash
# Round-3 call 4: same-box A/B of the smaller local-search kernel (out-of-line
# lane-serial matcher, rolled task loop, explicit DPP wave_sum) against HEAD;
# GA local-search section profile; the counter list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s4}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 900 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step listpmc 120 rocprofv3 -L
step abls_comp01 300 python -u tools/ab_ls.py comp01 8192 base small
step abls_med 300 python -u tools/ab_ls.py med 4096 base small
step ab_med 240 python -u tools/ab_eval.py med 65536 base:8 small:8
step ab_lg 240 python -u tools/ab_eval.py lg 65536 base:8 small:8
step ab_syn 300 python -u tools/ab_eval.py syn 262144 base:13 small:13
step lsprof_ga 300 python -u tools/ls_prof.py --config comp01 --pop 65536 --children 8192 --from-ga 0.6 --steps 1000
step lsprof_p1 300 python -u tools/ls_prof.py
step lsprof_p2 300 python -u tools/ls_prof.py --steps 1000 --pre-steps 3000
echo done
