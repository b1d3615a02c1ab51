#!/bin/bash
# Round-3 measurement call: LS and GA throughput after the redo-list change,
# the GA kernel trace, syn eval phase timings and PMC of the wide path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -u
export TMPDIR=/tmp
T=${1:-r03_prof}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 lim=$2; shift 2; echo "== $n"; timeout -k 10 $lim "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -c 600 $O/$n.log; echo; [ $rc -ge 124 ] && exit $rc; return 0; }
step ls200 300 python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 256
step ls1000 300 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 256
step ga8k 400 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 25 --min-seconds 1.0 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 512
step ga8k_trace 400 rocprofv3 --kernel-trace --stats -d $O/ga_trace -o run --output-format csv -- python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --gens 10 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --cpu-sample 0
step listpmc 120 rocprofv3 -L
step synvar 300 python -u tools/eval_variants.py syn 262144 13,77
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$(( ${i:-0} + 1 ))
  step pmcw$i 90 rocprofv3 --pmc $c --output-format csv -d $O/pmcw$i -o pmc -- python -u tools/eval_variants.py syn 65536 13
done
python tools/pmc_summary.py $O eval_lanes_kernel > $O/lanes.json; python tools/pmc_summary.py $O eval_corr_kernel > $O/corr.json
echo done
