#!/bin/bash
# Round-3 call 3: debug of the vector-memory lane phase (syn wide path), GA
# local-search section profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s3}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 1500 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step lsprof_ga 300 python -u tools/ls_prof.py --config comp01 --pop 65536 --children 8192 --from-ga 0.6 --steps 1000
echo done
