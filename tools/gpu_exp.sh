#!/bin/bash
# Eval parity tests, then variant timings (one gpurun call; profiling helper).
# usage: tools/gpu_exp.sh TAG "med-variants" "syn-variants"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-exp}
MEDV=${2:-8,1032}
SYNV=${3:-13}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "eval or syn or config" \
    --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/eval_variants.py med 65536 "$MEDV" > "$OUT/med.json" 2>"$OUT/err.log" || exit $?
timeout -k 10 200 python -u tools/eval_variants.py lg 65536 "$MEDV" > "$OUT/lg.json" 2>>"$OUT/err.log" || exit $?
timeout -k 10 300 python -u tools/eval_variants.py syn 262144 "$SYNV" > "$OUT/syn.json" 2>>"$OUT/err.log" || exit $?
cat "$OUT/med.json" "$OUT/lg.json" "$OUT/syn.json"
