#!/bin/bash
# Round-3 call 13: phase-2 student attendance masks in the local search
# (TT_LS_SMASK), tiled rank sort for replace / LPT order (TT_SORT_RANK) --
# GPU suite, same-box LS A/B, GA throughput and trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s13}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
bash tools/gpu_check.sh $T tests || exit $?
step abls_comp01 300 python -u tools/ab_ls.py comp01 8192 sm0 sm1
step abls_med 300 python -u tools/ab_ls.py med 4096 sm0 sm1
step abls_lg 300 python -u tools/ab_ls.py lg 4096 sm0 sm1
step ga8k 400 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 512
step ga8k_trace 400 rocprofv3 --kernel-trace --stats -d $O/ga_trace -o run --output-format csv -- python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0
echo done
