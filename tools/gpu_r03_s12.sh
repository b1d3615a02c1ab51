#!/bin/bash
# Round-3 call 12: sort kernels (constant-index in-thread steps, parallel order
# check) -- GA tests, GA throughput and trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s12}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step pytest_ga 400 python -u -m pytest tests/test_gpu_ga.py -m gpu -v --timeout 300 --timeout-method thread
step ga8k 400 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 512
step ga8k_trace 400 rocprofv3 --kernel-trace --stats -d $O/ga_trace -o run --output-format csv -- python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0
echo done
