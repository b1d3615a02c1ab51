# PMC passes over the wide eval path (syn instance, P = 65536, variant 13).
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcw}; mkdir -p $O
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc$i -o pmc -- python -u tools/eval_variants.py syn 65536 13 > $O/pmc$i.log 2>&1 || exit $?
done
python tools/pmc_summary.py $O eval_lanes_kernel > $O/lanes.json && python tools/pmc_summary.py $O eval_corr_kernel > $O/corr.json
