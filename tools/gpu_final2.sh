#!/bin/bash
# Round-end check: every GPU test, smoke, the bench line, then the phase-2 GA bench (8,192 and 32,768 children).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-final2}; O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_check.sh $T tests smoke bench || exit $?
grep -q " passed" $O/pytest_gpu.log && ! grep -q " failed" $O/pytest_gpu.log || exit 1
ARGS="--config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 64"
timeout -k 10 300 python -u tools/bench_ga.py $ARGS > $O/ga8k.log 2>&1 || exit $?
tail -1 $O/ga8k.log | grep -o '"gpu_children_per_s": [0-9.]*\|"feasible_fraction": [0-9.]*\|"children_per_s": [0-9.]*'
ARGS="--config comp01 --pop 65536 --children 32768 --gens 4 --steps 1000 --warm-gens 40 --warm-feasible 0.6 --cpu-sample 0"
timeout -k 10 300 python -u tools/bench_ga.py $ARGS > $O/ga32k.log 2>&1 || exit $?
tail -1 $O/ga32k.log | grep -o '"gpu_children_per_s": [0-9.]*\|"feasible_fraction": [0-9.]*'
timeout -k 10 300 python -u tools/bench_ls.py --pop 4096 --steps 200 > $O/ls200.log 2>&1 || exit $?
tail -1 $O/ls200.log
timeout -k 10 300 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 256 > $O/ls1000.log 2>&1 || exit $?
tail -1 $O/ls1000.log
