# rocprof kernel stats of the full-GA bench (comp01, pop 65536) and of the LS bench; PMC of the LS kernel.
set -u
export TMPDIR=/tmp
O=gpurun_out/pga; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ga -o run --output-format csv -- python -u tools/bench_ga.py --config comp01 --gens 2 --cpu-sample 64 > $O/ga.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ls -o run --output-format csv -- python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 64 > $O/ls.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM --output-format csv -d $O/pmc1 -o pmc -- python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 16 > $O/pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d $O/pmc2 -o pmc -- python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 16 > $O/pmc2.log 2>&1 || exit $?
python tools/pmc_summary.py $O local_search > $O/ls_pmc.json
tail -1 $O/ga.log; tail -1 $O/ls.log
