#!/bin/bash
# Round-3 call 18: lazy old-slot task in the phase-1 Move1 loop (TT_LS_LAZY1) --
# LS and GA tests, same-box LS A/B, GA throughput per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s18}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
bash tools/gpu_check.sh $T tests || exit $?
step abls_comp01 300 python -u tools/ab_ls.py comp01 8192 lz0 lz1
step abls_med 300 python -u tools/ab_ls.py med 4096 lz0 lz1
step abls_lg 300 python -u tools/ab_ls.py lg 4096 lz0 lz1
for v in lz0 lz1; do
step ga8k_$v 300 python -u tools/bench_ga.py --lib ab_libs/libttga_$v.so --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0
done
echo done
