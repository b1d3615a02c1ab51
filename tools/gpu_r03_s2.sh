#!/bin/bash
# Round-3 call 2: statistical GA comparison (device side), same-box A/B of the
# local-search and wide-eval changes against 3bd2de9, LS/GA throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_s2}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 700 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step gaq_med 300 python -u tools/ga_quality_program.py device --ref profiles/r03_ga_refprog_med.json --out $O/ga_quality_med.json
step gaq_comp01 300 python -u tools/ga_quality_program.py device --ref profiles/r03_ga_refprog_comp01.json --out $O/ga_quality_comp01.json
step ab_med 240 python -u tools/ab_eval.py med 65536 head:8 lean:8
step ab_lg 240 python -u tools/ab_eval.py lg 65536 head:8 lean:8
step ab_syn 300 python -u tools/ab_eval.py syn 262144 head:13 lanesvm:13 lean:13 corrold:13 before:13
step abls_comp01 300 python -u tools/ab_ls.py comp01 8192 before head noslp
step abls_med 300 python -u tools/ab_ls.py med 4096 before head noslp
step ls200 300 python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 256
step ls1000 300 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 256
step ga8k 400 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 512
echo done
