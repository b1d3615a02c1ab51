#!/bin/bash
# Round-3 call 5: same-box A/B of the local-search visit row prefetch and the
# phase-1 Move1 trial window against HEAD; GA section profile; icache counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s5}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 700 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step abls_comp01 300 python -u tools/ab_ls.py comp01 8192 base2 pref m1win
step abls_med 300 python -u tools/ab_ls.py med 4096 base2 pref m1win
step abls_lg 300 python -u tools/ab_ls.py lg 4096 base2 m1win
step lsprof_ga 300 python -u tools/ls_prof.py --config comp01 --pop 65536 --children 8192 --from-ga 0.6 --steps 1000
step pmc_icache 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --output-format csv -d $O/pmc_icache -o pmc -- python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 0
echo done
