#!/bin/bash
# GA/LS parity tests, then the phase-2 GA bench (comp01, pop 65,536, 8,192
# children per generation, maxSteps 1000) and its rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ga}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
ARGS="--config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6"
timeout -k 10 400 python -u tools/bench_ga.py $ARGS --cpu-sample 64 > "$OUT/ga_c8k.log" 2>&1 || exit $?
tail -1 "$OUT/ga_c8k.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python -u tools/bench_ga.py $ARGS --cpu-sample 0 > "$OUT/ga_prof.log" 2>&1 || exit $?
head -8 "$OUT/prof/run_kernel_stats.csv" | cut -c1-160
