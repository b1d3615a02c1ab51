#!/bin/bash
# Same-box A/B of localSearch builds in ab_libs/ (tools/ab_ls.py), two instances.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-abls}; shift; mkdir -p $O
timeout -k 10 400 python -u tools/ab_ls.py comp01 8192 "$@" > $O/comp01.json 2> $O/comp01.err || exit $?
cat $O/comp01.json
timeout -k 10 400 python -u tools/ab_ls.py med 4096 "$@" > $O/med.json 2> $O/med.err || exit $?
cat $O/med.json
