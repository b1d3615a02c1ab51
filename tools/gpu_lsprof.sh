#!/bin/bash
# Section profile of the local search (profiling build): phase 1 from random init and phase 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-lsprof}; mkdir -p $O
timeout -k 10 300 python -u tools/ls_prof.py > $O/phase1.json 2> $O/phase1.err || exit $?
timeout -k 10 300 python -u tools/ls_prof.py --steps 1000 --pre-steps 3000 > $O/phase2.json 2> $O/phase2.err || exit $?
timeout -k 10 300 python -u tools/ls_prof.py --config comp01 --pop 65536 --children 8192 --from-ga 0.6 --steps 1000 > $O/ga.json 2> $O/ga.err || exit $?
tail -c 1500 $O/phase1.json
