#!/bin/bash
# Round-3 call 6: same-box A/B of the phase-1 Move1 window without the row
# prefetch; the GPU suite, smoke, bench and LS/GA throughput on the new tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s6}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 700 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step abls_comp01 300 python -u tools/ab_ls.py comp01 8192 base2 m1win win
step abls_med 300 python -u tools/ab_ls.py med 4096 base2 m1win win
step abls_lg 300 python -u tools/ab_ls.py lg 4096 base2 win
bash tools/gpu_check.sh $T tests smoke bench || exit $?
step ls200 300 python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 256
step ls1000 300 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 256
step ga8k 400 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 512
echo done
