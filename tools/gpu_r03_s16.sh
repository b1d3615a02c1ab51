#!/bin/bash
# Round-3 call 16: measurement refresh after the sort / matcher / copy changes --
# GPU suite, smoke, headline bench + kernel trace, syn bench, LS and GA benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s16}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
bash tools/gpu_check.sh $T tests smoke bench prof benchsyn || exit $?
step ls200 300 python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 256
step ls1000 300 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 256
step ga8k 300 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 512
step ga32k 300 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 32768 --gens 10 --min-seconds 1.0 --steps 1000 --warm-gens 30 --warm-feasible 0.6 --cpu-sample 0
echo done
