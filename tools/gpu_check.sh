#!/bin/bash
# GPU checks for one gpurun call. Each step runs under its own time limit and
# the script stops at the first timeout / abort / crash (exit >= 124); test
# failures (exit 1) do not stop the later measurement steps.
# usage: tools/gpu_check.sh [tag] [steps...]   steps: tests smoke bench prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}; shift || true
STEPS=${*:-tests smoke bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {
    local name=$1 limit=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    gatests) run pytest_ga 600 python -u -m pytest tests/test_gpu_ga.py -m gpu -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python -u bench.py ;;
    benchsyn) run bench_syn 600 python -u bench.py --config syn --pop 262144 --steps 10 --warmup 2 ;;
    profsyn) run rocprof_syn 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_syn" -o run --output-format csv -- python -u bench.py --config syn --pop 262144 --no-pmc --no-cpu --steps 10 --warmup 2 ;;
    benchlg) run bench_lg 600 python -u bench.py --config lg --steps 100 ;;
    phases) run phases 300 python -u tools/eval_variants.py med 65536 8,24,40,72,136,264,520 ;;
    quality) run ga_quality 900 python -u tools/ga_quality.py --config sm --seeds 16 --gens 2001 --steps 200 --out "$OUT/ga_quality_sm.json" ;;
    ls)    run bench_ls 600 python -u tools/bench_ls.py --pop 4096 --steps 200 ;;
    ls1000) run bench_ls1000 600 python -u tools/bench_ls.py --pop 4096 --steps 1000 --cpu-sample 256 ;;
    listpmc) run listpmc 120 rocprofv3 -L ;;
    pmc1)  run pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmc1" -o pmc -- python -u bench.py --no-pmc --no-cpu --steps 3 --warmup 1 ;;
    pmc2)  run pmc2 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc2" -o pmc -- python -u bench.py --no-pmc --no-cpu --steps 3 --warmup 1 ;;
    pmc3)  run pmc3 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc3" -o pmc -- python -u bench.py --no-pmc --no-cpu --steps 3 --warmup 1 ;;
    pmc4)  run pmc4 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc4" -o pmc -- python -u bench.py --no-pmc --no-cpu --steps 3 --warmup 1 ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python -u bench.py --no-pmc --no-cpu --steps 100 ;;
  esac
done
echo "done"
