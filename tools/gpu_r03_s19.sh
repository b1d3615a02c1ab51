#!/bin/bash
# Round-3 call 19: possibleRooms prefetch in the register matcher (A/B, parity),
# GA kernel trace in the steady regime (300 untimed generations first, then 20
# traced ones at >= 99.9 % feasible).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s19}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step pytest_rooms 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ga.py -m gpu -v --timeout 200 --timeout-method thread
step abrooms_comp01 200 python -u tools/ab_rooms.py comp01 8192 mpf0 mpf1 mt1
step abrooms_med 200 python -u tools/ab_rooms.py med 8192 mpf0 mpf1 mt1
step ga8k_steady_trace 400 rocprofv3 --kernel-trace --stats -d $O/ga_trace -o run --output-format csv -- python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 20 --steps 1000 --warm-gens 300 --warm-feasible 1.1 --cpu-sample 0
echo done
