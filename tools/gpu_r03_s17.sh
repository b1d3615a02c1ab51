#!/bin/bash
# Round-3 call 17: room-assignment parity (register-matcher limits), GA
# children's local-search section profile, LS occupancy A/B (waves per EU 4/5/6)
# at the GA's child count and in the GA itself.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s17}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step pytest_rooms 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "assign_rooms or random_init"
step lsprof_ga 300 python -u tools/ls_prof.py --config comp01 --pop 65536 --children 8192 --from-ga 0.6 --steps 1000
step abls_comp01 300 python -u tools/ab_ls.py comp01 8192 wpe5 wpe4 wpe6
for v in wpe5 wpe4 wpe6; do
step ga8k_$v 300 python -u tools/bench_ga.py --lib ab_libs/libttga_$v.so --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0
done
echo done
