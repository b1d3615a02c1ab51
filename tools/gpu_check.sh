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
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python -u bench.py ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python -u bench.py --no-cpu --steps 100 ;;
  esac
done
echo "done"
