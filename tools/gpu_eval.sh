#!/bin/bash
# Eval parity tests then variant timing (profiling helper; one gpurun call).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ev}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "eval or syn" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
# wide path at the scaling size; 13|16 skips eval_corr's build phase, 13|32 its corr phase (timing only)
timeout -k 10 200 python -u tools/eval_variants.py syn 262144 13,29,45 > "$OUT/variants_syn.json" 2>"$OUT/err.log"; rc=$?
cat "$OUT/variants_syn.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/eval_variants.py med 65536 8,7,13 > "$OUT/variants_med.json" 2>>"$OUT/err.log"; rc=$?
cat "$OUT/variants_med.json"; exit $rc
