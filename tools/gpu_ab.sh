#!/bin/bash
# Same-box A/B of eval builds in ab_libs/ (tools/ab_build.sh); one gpurun call.
# usage: tools/gpu_ab.sh TAG CONFIG P spec...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/ab_eval.py "$@" > "$OUT/ab_$1.json" 2>"$OUT/err_$1.log"; rc=$?
cat "$OUT/ab_$1.json"; tail -3 "$OUT/err_$1.log"; exit $rc
