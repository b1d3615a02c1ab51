#!/bin/bash
# LS/GA parity tests, then the same-box LS A/B (old vs new) and the phase-2 GA bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-ls2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "local_search or island or ordered or driver or ls" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_abls.sh ${1:-ls2} old new || exit $?
ARGS="--config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0"
timeout -k 10 300 python -u tools/bench_ga.py $ARGS > $O/ga8k.log 2>&1 || exit $?
tail -1 $O/ga8k.log | grep -o '"gpu_children_per_s": [0-9.]*\|"feasible_fraction": [0-9.]*'
ARGS="--config comp01 --pop 65536 --children 32768 --gens 4 --steps 1000 --warm-gens 40 --warm-feasible 0.6 --cpu-sample 0"
timeout -k 10 300 python -u tools/bench_ga.py $ARGS > $O/ga32k.log 2>&1 || exit $?
tail -1 $O/ga32k.log | grep -o '"gpu_children_per_s": [0-9.]*\|"feasible_fraction": [0-9.]*'
