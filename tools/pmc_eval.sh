set -u
export TMPDIR=/tmp
O=gpurun_out/$1; V=$2; mkdir -p $O
timeout -k 10 200 python -u tools/eval_variants.py med 65536 $V,$((V|16)),$((V|32)),$((V|64)),$((V|48)) > $O/phases.json 2>$O/err.log || exit $?
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc$i -o pmc -- python -u tools/eval_variants.py med 65536 $V > $O/pmc$i.log 2>&1 || exit $?
done
cat $O/phases.json
