# PMC passes over the local-search kernel (bench_ls workload; extra args go to bench_ls.py).
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcls}; shift || true
mkdir -p $O
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc$i -o pmc -- python -u tools/bench_ls.py --cpu-sample 0 --reps 1 "$@" > $O/pmc$i.log 2>&1 || exit $?
done
python tools/pmc_summary.py $O local_search_kernel > $O/ls.json
