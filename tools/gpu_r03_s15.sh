#!/bin/bash
# Round-3 call 15: register-resident lane matcher (TT_MATCH_REG) for room
# assignment / mutation; population-aware student-mask gate -- GPU suite,
# same-box A/B of the room kernels, GA throughput per variant, GA trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s15}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
bash tools/gpu_check.sh $T tests || exit $?
step abrooms_comp01 200 python -u tools/ab_rooms.py comp01 8192 mreg0 mreg1
step abrooms_med 200 python -u tools/ab_rooms.py med 8192 mreg0 mreg1
step abrooms_lg 200 python -u tools/ab_rooms.py lg 8192 mreg0 mreg1
step abls_med4k 300 python -u tools/ab_ls.py med 4096 mreg0 mreg1
for v in mreg0 mreg1; do
step ga8k_$v 300 python -u tools/bench_ga.py --lib ab_libs/libttga_$v.so --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0
done
step ga8k_trace 400 rocprofv3 --kernel-trace --stats -d $O/ga_trace -o run --output-format csv -- python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0
echo done
