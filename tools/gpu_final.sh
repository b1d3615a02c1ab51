#!/bin/bash
# Round-end evidence in one gpurun call: GPU tests, smoke, headline bench +
# rocprof, syn/lg bench lines, tile5 PMC passes, LS benches, phase-2 GA bench
# with its rocprof kernel stats. Every step has its own time limit; the script
# stops at the first timeout / crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-final}; O=gpurun_out/$TAG; mkdir -p $O
run() {
    local name=$1 limit=$2; shift 2
    echo "== $name"
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 "$O/$name.log" | cut -c1-300
    if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
    return 0
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python -u bench.py
run rocprof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python -u bench.py --no-pmc --no-cpu --steps 100
run bench_syn 600 python -u bench.py --config syn --pop 262144 --steps 20 --warmup 3
run rocprof_syn 600 rocprofv3 --kernel-trace --stats -d $O/prof_syn -o run --output-format csv -- python -u bench.py --config syn --pop 262144 --no-pmc --no-cpu --steps 10 --warmup 2
run bench_lg 600 python -u bench.py --config lg --steps 200
run bench_ls 600 python -u tools/bench_ls.py --pop 4096 --steps 200
run bench_ls2 600 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 256
run ga_prof 600 rocprofv3 --kernel-trace --stats -d $O/prof_ga -o run --output-format csv -- python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0
echo done
