#!/bin/bash
# GA parity tests, then the phase-2 GA bench (comp01, pop 65,536, 8,192 children, LPT dispatch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ga2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
ARGS="--config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6"
timeout -k 10 400 python -u tools/bench_ga.py $ARGS --cpu-sample 64 > $O/ga_c8k.log 2>&1 || exit $?
tail -1 $O/ga_c8k.log | cut -c1-400
