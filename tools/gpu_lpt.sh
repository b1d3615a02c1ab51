#!/bin/bash
# LPT A/B for the phase-2 GA bench (8,192 and 32,768 children) after the GA/LS parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
O=gpurun_out/s3lpt; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py tests/test_gpu_parity.py -x -q -k "island or ordered or local_search or breed or replace" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
ARGS="--config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0"
for l in off on; do timeout -k 10 300 python -u tools/bench_ga.py $ARGS --lpt $l > $O/ga_$l.log 2>&1 || exit $?; tail -1 $O/ga_$l.log | grep -o '"lpt_dispatch": [a-z]*\|"gpu_children_per_s": [0-9.]*\|"feasible_fraction": [0-9.]*'; done
ARGS="--config comp01 --pop 65536 --children 32768 --gens 4 --steps 1000 --warm-gens 40 --warm-feasible 0.6 --cpu-sample 0"
for l in off on; do timeout -k 10 300 python -u tools/bench_ga.py $ARGS --lpt $l > $O/ga32_$l.log 2>&1 || exit $?; tail -1 $O/ga32_$l.log | grep -o '"lpt_dispatch": [a-z]*\|"gpu_children_per_s": [0-9.]*\|"feasible_fraction": [0-9.]*'; done
