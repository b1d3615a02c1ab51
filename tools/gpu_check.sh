#!/bin/bash
# GPU checks for one gpurun call. Each step runs under its own time limit and
# the script stops at the first timeout / abort / crash (exit >= 124); test
# failures (exit 1) do not stop the later measurement steps.
# usage: tools/gpu_check.sh [tag] [steps...]
#   tests gatests derive smoke bench prof benchsyn profsyn benchlg phases quality
#   ls ls1000 ga8k ga32k gatrace lsprof timeprob profderive pmcderive listpmc
#   stamps replace ablanes pmc1..pmc4 (headline eval) pmcls (phase-2 local search) pmcga (GA children's
#   local search) pmcwide (syn wide path) abls abeval
#   round 5: gaabx / ablsx (GA / LS A/B of ab_libs/libttga_$LIBS, configs in GACFGS / LSCFGS),
#   gaisl (bench_ga --islands $ISLS), isltests, gacomps20 / gacomps20i2 (20-comp tables, 1 / 2
#   islands), lstail / lsprofc (LS launch tail and section profiles, profiling library),
#   occprobe / occsweep (tools/occ_probe: resident waves against LDS and scratch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04}; shift || true
STEPS=${*:-tests smoke bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {
    local name=$1 limit=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -c 700 "$OUT/$name.log"; echo
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
# PMC passes of one command, each pass its own run (rocprofv3 does not split
# counters over passes); summary by tools/pmc_summary.py for kernel $2
PASS1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
PASS2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
PASS3="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU"
pmc() {
    local name=$1 kernel=$2; shift 2
    local i=0 c
    for c in "$PASS1" "$PASS2" "$PASS3"; do
        i=$((i + 1))
        echo "== $name pass $i"
        timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$OUT/$name/pmc$i" -o pmc -- "$@" \
            > "$OUT/$name.pmc$i.log" 2>&1 || { echo "pmc pass $i rc=$?"; exit 125; }
    done
    python tools/pmc_summary.py "$OUT/$name" "$kernel" ${PMC_LAST:+--last $PMC_LAST} > "$OUT/$name.json"; cat "$OUT/$name.json"
}
# the profiling library (make prof) must be newer than every source it is built from
prof_fresh() {
    local lib=timetabling-ga-mpi-openmp_amd/libttga_prof.so
    if [ ! -f "$lib" ] || [ -n "$(find timetabling-ga-mpi-openmp_amd/csrc include -newer "$lib" -type f)" ]; then
        echo "stale $lib: run make -C timetabling-ga-mpi-openmp_amd prof"; exit 2
    fi
}
GA8K="--config comp01 --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6"
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    widetests) run pytest_wide 900 python -u -m pytest tests/test_gpu_wide_rooms.py -m gpu -v --timeout 300 --timeout-method thread ;;
    r6tests) run pytest_r6 1000 python -u -m pytest tests/test_gpu_wide_rooms.py tests/test_gpu_bench.py tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "wide_rooms or syn_sample or bench or mask_policy" ;;
    stagtests) run pytest_stag 900 python -u -m pytest tests/test_gpu_ga.py -m gpu -v --timeout 300 --timeout-method thread -k "staggered or island_generations or breed_vs or replace_vs" ;;
    gastag) for c in ${STAGCFGS:-comp15 comp16 comp10 comp01}; do for sch in ${STAGSCH:-batch staggered}; do for np in ${STAGPARTS:-2}; do run ga8k_${c}_${sch}_$np 400 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample ${CPUS:-0} --schedule $sch --parts $np; done; done; done ;;
    lsroof) run ls_roofline 1100 python -u tools/ls_roofline.py ${LSROOF:---config comp01 --config comp10 --config comp15} --out "$OUT/ls_roofline.jsonl" ;;
    gacomps20s) run ga_comps20_stag 1100 python -u tools/ga_comps.py "$OUT/ga_comps20_staggered.json" --schedule staggered ;;
    qualstag) run ga_quality_sm_stag 600 python -u tools/ga_quality.py --config sm --seeds 16 --gens 2001 --steps 200 --device-children 2 --device-gens 1000 --device-schedule staggered --out "$OUT/ga_quality_sm_staggered.json" &&
              run ga_quality_med_stag 900 python -u tools/ga_quality.py --config med --seeds 16 --gens 2001 --steps 1000 --device-children 2 --device-gens 1000 --device-schedule staggered --no-ref-as-is --out "$OUT/ga_quality_med_staggered.json" ;;
    t5parts) run t5_components 600 python -u tools/t5_components.py ab_libs/libttga_abl.so med 65536 ;;
    abt5x) for c in ${T5CFGS:-med lg comp01 med}; do run ab_t5_$c 300 python -u tools/ab_eval.py $c 65536 $T5SPECS; done ;;
    stagtrace) for sch in batch staggered; do n=20; [ $sch = staggered ] && n=40
                 run trace_$sch 400 rocprofv3 --kernel-trace -d "$OUT/tr_$sch" -o run --output-format csv -- python -u tools/bench_ga.py --config ${TRCFG:-comp20} --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 20 --cpu-sample 0 --schedule $sch &&
                 python tools/trace_window.py "$OUT/tr_$sch/run_kernel_trace.csv" $n > "$OUT/trace_window_$sch.json" && python tools/trace_overlap.py "$OUT/tr_$sch/run_kernel_trace.csv" --last $n > "$OUT/trace_overlap_$sch.json"; done ;;
    stagl) for c in ${STAGCFGS:-comp20 comp15}; do for l in on off; do run ga8k_${c}_stag_lpt$l 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --schedule staggered --lpt $l; done; run ga8k_${c}_batch 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0; done ;;
    lsevaltests) run pytest_lseval 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ga.py tests/test_gpu_configs.py tests/test_gpu_baseline_configs.py tests/test_gpu_wide_rooms.py -m gpu -q --timeout 300 --timeout-method thread ;;
    abrooms) for c in ${ROOMCFGS:-syn:65536 comp01:65536 med:65536 lg:65536}; do run ab_rooms_${c%%:*} 300 python -u tools/ab_rooms.py ${c%%:*} ${c##*:} ${LIBS:-rw0 rw1}; done ;;
    roomroof) run rooms_roofline 900 python -u tools/rooms_roofline.py ${ROOMROOF:---config syn:65536 --config comp01:65536} --lib ${ROOMLIB:-tree} --out "$OUT/rooms_roofline.jsonl" ;;
    benchtests) run pytest_bench 600 python -u -m pytest tests/test_gpu_bench.py -m gpu -v --timeout 300 --timeout-method thread ;;
    gastagab) for i in 1 2; do for c in ${GACFGS:-comp15 comp16 comp01}; do for sch in ${STAGSCH:-staggered}; do for l in $LIBS; do run ga8k_${c}_${sch}_${l}_$i 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --schedule $sch --lib ab_libs/libttga_$l.so; done; done; done; done ;;
    gatests) run pytest_ga 600 python -u -m pytest tests/test_gpu_ga.py -m gpu -v --timeout 300 --timeout-method thread ;;
    derive) run pytest_derive 400 python -u -m pytest tests/test_gpu_derive.py -m gpu -v --timeout 200 --timeout-method thread ;;
    newtests) run pytest_new 600 python -u -m pytest tests/test_gpu_derive.py tests/test_gpu_ga.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "derive or derived or permutation or redo" ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python -u bench.py ;;
    benchsyn) run bench_syn 600 python -u bench.py --config syn --pop 262144 --steps 10 --warmup 2 ;;
    profsyn) run rocprof_syn 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_syn" -o run --output-format csv -- python -u bench.py --config syn --pop 262144 --no-pmc --no-cpu --steps 10 --warmup 2 ;;
    benchlg) run bench_lg 600 python -u bench.py --config lg --steps 100 ;;
    phases) run phases 300 python -u tools/eval_variants.py med 65536 8,24,40,72,136,264,520 ;;
    quality) run ga_quality 900 python -u tools/ga_quality.py --config sm --seeds 16 --gens 2001 --steps 200 --out "$OUT/ga_quality_sm.json" ;;
    ls)    run bench_ls 300 python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 256 ;;
    ls1000) run bench_ls1000 300 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 256 ;;
    ga8k)  run ga8k 400 python -u tools/bench_ga.py $GA8K --gens 25 --min-seconds 1.0 --cpu-sample 512 ;;
    ga32k) run ga32k 300 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 32768 --gens 10 --min-seconds 1.0 --steps 1000 --warm-gens 30 --warm-feasible 0.6 --cpu-sample 0 ;;
    gacomps) for c in comp05 comp10 comp15 comp20; do run ga8k_$c 400 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 512; done ;;
    abgate) run abgate_med 400 python -u tools/ab_ls.py med 4096 g1 g2 g3 g4 && run abgate_comp01 400 python -u tools/ab_ls.py comp01 8192 g1 g2 g3 g4 &&
            for c in comp15 comp10 comp01; do for l in g1 g2 g3 g4; do run gagate_${c}_$l 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done ;;
    gasteady) run ga8k_steady_trace 500 rocprofv3 --kernel-trace -d "$OUT/ga_steady" -o run --output-format csv -- python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --steps 1000 --warm-gens 400 --warm-feasible 0.999 --gens 20 --cpu-sample 0 &&
              python tools/trace_window.py "$OUT/ga_steady/run_kernel_trace.csv" 20 > "$OUT/ga_steady_window.json"; cat "$OUT/ga_steady_window.json" ;;
    gatrace) run ga8k_trace 400 rocprofv3 --kernel-trace --stats -d "$OUT/ga_trace" -o run --output-format csv -- python -u tools/bench_ga.py $GA8K --gens 20 --cpu-sample 0 ;;
    lsprof) prof_fresh; run lsprof_ga 300 python -u tools/ls_prof.py --config comp01 --pop 65536 --children 8192 --from-ga 0.999 --steps 1000 ;;
    timeprob) run time_problem 600 python -u tools/time_problem.py "$OUT/time_problem.json" 5 ;;
    profderive) run rocprof_derive 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_derive" -o run --output-format csv -- python -u tools/time_problem.py "$OUT/time_problem_traced.json" 5 ;;
    pmcderive)
        for c in "SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_LDS"; do
            i=$(( ${i:-0} + 1 ))
            run pmc_derive$i 150 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_derive/p$i" -o pmc -- python -u tools/time_problem.py "$OUT/time_problem_pmc$i.json" 3 syn
        done
        python tools/pmc_summary.py "$OUT/pmc_derive" derive_corr_kernel > "$OUT/pmc_derive.json"; cat "$OUT/pmc_derive.json" ;;
    listpmc) run listpmc 120 rocprofv3 -L ;;
    pmc1)  run pmc1 120 rocprofv3 --pmc $PASS1 --output-format csv -d "$OUT/pmc1" -o pmc -- python -u bench.py --no-pmc --no-cpu --steps 3 --warmup 1 ;;
    pmc2)  run pmc2 120 rocprofv3 --pmc $PASS2 --output-format csv -d "$OUT/pmc2" -o pmc -- python -u bench.py --no-pmc --no-cpu --steps 3 --warmup 1 ;;
    pmc3)  run pmc3 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc3" -o pmc -- python -u bench.py --no-pmc --no-cpu --steps 3 --warmup 1 ;;
    pmc4)  run pmc4 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc4" -o pmc -- python -u bench.py --no-pmc --no-cpu --steps 3 --warmup 1 ;;
    pmcls) pmc pmc_ls local_search_kernel python -u tools/bench_ls.py --cpu-sample 0 --reps 1 --pop 4096 --steps 1000 --pre-steps 3000 ;;
    pmcga) PMC_LAST=10 pmc pmc_ga local_search_kernel python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --steps 1000 --warm-gens 400 --warm-feasible 0.999 --gens 10 --cpu-sample 0 ;;
    pmcwide) pmc pmc_wide eval_lanes python -u tools/eval_variants.py syn 65536 13 &&
             python tools/pmc_summary.py "$OUT/pmc_wide" eval_corr > "$OUT/pmc_wide_corr.json" ;;
    abls)  run ab_comp01 400 python -u tools/ab_ls.py comp01 8192 old new && run ab_med 400 python -u tools/ab_ls.py med 4096 old new ;;
    stamps) prof_fresh; run t5_stamps 300 python -u tools/t5_stamps.py --raw "$OUT/t5_stamps_raw.npz" ;;
    replace) run time_replace 300 python -u tools/time_replace.py ;;
    ablanes) run ab_lanes 400 python -u tools/ab_eval.py syn 262144 gap0:13 gap1:13 gap0:77 gap1:77 ;;
    abhot) run ab_hot_comp01 400 python -u tools/ab_ls.py comp01 8192 hot0 hot1 hot2 && run ab_hot_med 400 python -u tools/ab_ls.py med 4096 hot0 hot1 hot2 ;;
    gahot) for i in 1 2; do run ga8k_hot0_$i 300 python -u tools/bench_ga.py $GA8K --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_hot0.so; run ga8k_hot1_$i 300 python -u tools/bench_ga.py $GA8K --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_hot1.so; run ga8k_hot2_$i 300 python -u tools/bench_ga.py $GA8K --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_hot2.so; done ;;
    abocc) run ab_occ_med 300 python -u tools/ab_eval.py med 65536 t5old:8 t5old:7 occ:8 occ:7 && run ab_occ_lg 300 python -u tools/ab_eval.py lg 65536 t5old:8 t5old:7 occ:8 occ:7 && run ab_occ_comp01 300 python -u tools/ab_eval.py comp01 65536 t5old:8 occ:8 occ:7 ;;
    abeval) run ab_eval 300 python -u tools/ab_eval.py old new ;;
    abt5) run ab_t5_med 300 python -u tools/ab_eval.py med 65536 old:8 new:8 old:7 new:7 && run ab_t5_lg 300 python -u tools/ab_eval.py lg 65536 old:8 new:8 && run ab_t5_comp01 300 python -u tools/ab_eval.py comp01 65536 old:8 new:8 && run ab_t5_med2 300 python -u tools/ab_eval.py med 65536 new:8 old:8 ;;
    abcorr) run ab_corr_syn 400 python -u tools/ab_eval.py syn 262144 old:13 new:13 && run ab_corr_med 300 python -u tools/ab_eval.py med 65536 old:8 new:8 ;;
    valurate) run valu_rate 120 tools/valu_rate ;;
    abls4) run ab4_comp01 400 python -u tools/ab_ls.py comp01 8192 old new noscv norow && run ab4_med 400 python -u tools/ab_ls.py med 4096 old new noscv norow ;;
    gaab4) for i in 1 2; do for l in old new noscv norow; do run ga8k_${l}_$i 300 python -u tools/bench_ga.py $GA8K --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done ;;
    gaab) for i in 1 2; do for l in old new; do run ga8k_${l}_$i 300 python -u tools/bench_ga.py $GA8K --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done ;;
    abr5) run ab_r5_syn 400 python -u tools/ab_eval.py syn 262144 r4:13 r5a:13 r4:13 r5a:13 && run ab_r5_med 300 python -u tools/ab_eval.py med 65536 r4:8 r5a:8 ;;
    lsprofc) prof_fresh; for c in comp15 comp10; do run lsprof_ga_$c 400 python -u tools/ls_prof.py --config $c --pop 65536 --children 8192 --from-ga 0.6 --warm-gens 96 --steps 1000; done ;;
    pmcgac) for c in comp15 comp10; do PMC_LAST=10 pmc pmc_ga_$c local_search_kernel python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 10 --cpu-sample 0; done ;;
    abr5b) run ab_r5b_syn 400 python -u tools/ab_eval.py syn 262144 r4:13 r5b:13 r4:13 r5b:13 &&
           run ab_r5b_med 300 python -u tools/ab_eval.py med 65536 r4:8 r5b:8 r5b:9 r4:8 r5b:9 &&
           run ab_r5b_lg 300 python -u tools/ab_eval.py lg 65536 r4:8 r5b:9 r4:8 r5b:9 &&
           run ab_r5b_comp01 300 python -u tools/ab_eval.py comp01 65536 r4:8 r5b:9 r4:8 r5b:9 ;;
    gap1b) for c in comp15 comp10 comp01; do for l in r5b0 r5b; do run ga8k_${c}_$l 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done &&
           run ga8k_comp15_check 300 python -u tools/bench_ga.py --config comp15 --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 512 ;;
    lstests) run pytest_ls 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ga.py tests/test_gpu_configs.py tests/test_gpu_baseline_configs.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
    gap1c) for i in 1 2; do for c in comp15 comp10 comp05 comp01; do for l in r5c0 r5c; do run ga8k_${c}_${l}_$i 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done; done ;;
    gap1d) for i in 1 2; do for c in comp15 comp10 comp05 comp01; do for l in r5d0 r5d; do run ga8k_${c}_${l}_$i 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done; done ;;
    abt5d) run ab_t5d_med 300 python -u tools/ab_eval.py med 65536 r5d:8 prio:8 r5d:9 r5d:8 prio:8 r5d:9 &&
           run ab_t5d_lg 300 python -u tools/ab_eval.py lg 65536 r5d:8 prio:8 r5d:9 r5d:8 prio:8 r5d:9 &&
           run ab_t5d_comp01 300 python -u tools/ab_eval.py comp01 65536 r5d:8 prio:8 r5d:9 r5d:8 prio:8 r5d:9 ;;
    abprio) run ab_prio_med 400 python -u tools/ab_eval.py med 65536 r5e:8 pA:8 pB:8 pC:8 pD:8 pE:8 r5e:8 pA:8 pB:8 pC:8 pD:8 pE:8 &&
            run ab_prio_lg 400 python -u tools/ab_eval.py lg 65536 r5e:8 pA:8 pB:8 pC:8 pD:8 pE:8 r5e:8 pA:8 pB:8 pC:8 pD:8 pE:8 &&
            run ab_prio_comp01 400 python -u tools/ab_eval.py comp01 65536 r5e:8 pA:8 pB:8 pC:8 pD:8 pE:8 r5e:8 pA:8 pB:8 pC:8 pD:8 pE:8 ;;
    ga01off) for i in 1 2; do for l in r5e p1boff; do run ga8k_comp01_${l}_$i 300 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done ;;
    lsprof01) for l in profon profoff; do run lsprof_comp01_$l 300 python -u tools/ls_prof.py --config comp01 --pop 65536 --children 8192 --from-ga 0.999 --steps 1000 --lib ab_libs/libttga_$l.so; done ;;
    abprio2) run ab_prio2_med 400 python -u tools/ab_eval.py med 65536 r5f:8 pG:8 pH:8 pI:8 r5f:8 pG:8 pH:8 pI:8 &&
             run ab_prio2_lg 400 python -u tools/ab_eval.py lg 65536 r5f:8 pG:8 pH:8 pI:8 r5f:8 pG:8 pH:8 pI:8 &&
             run ab_prio2_comp01 400 python -u tools/ab_eval.py comp01 65536 r5f:8 pG:8 pH:8 pI:8 r5f:8 pG:8 pH:8 pI:8 ;;
    gap1f) for i in 1 2; do for c in comp15 comp10 comp01; do for l in r5f0 r5f; do run ga8k_${c}_${l}_$i 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done; done ;;
    gap1g) for i in 1 2; do for c in comp15 comp10 comp01; do for l in r5g0 r5g; do run ga8k_${c}_${l}_$i 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done; done ;;
    gap1h) for i in 1 2; do for c in comp01 comp15; do for l in r5g0 r5g r5h; do run ga8k_${c}_${l}_$i 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done; done ;;
    abgrid) run ab_grid_med 300 python -u tools/ab_eval.py med 65536 r5g:8 r5g:1032 r5g:7 r5g:9 r5g:8 r5g:1032 r5g:7 r5g:9 &&
            run ab_grid_lg 300 python -u tools/ab_eval.py lg 65536 r5g:8 r5g:1032 r5g:7 r5g:9 r5g:8 r5g:1032 r5g:7 r5g:9 ;;
    abgrid2) run ab_grid2_med 300 python -u tools/ab_eval.py med 65536 r5j:8 r5j:2056 r5j:8 r5j:2056 &&
             run ab_grid2_lg 300 python -u tools/ab_eval.py lg 65536 r5j:8 r5j:2056 r5j:8 r5j:2056 &&
             run ab_grid2_comp01 300 python -u tools/ab_eval.py comp01 65536 r5j:8 r5j:2056 r5j:8 r5j:2056 &&
             run ab_grid2_med262k 300 python -u tools/ab_eval.py med 262144 r5j:8 r5j:2056 r5j:8 r5j:2056 &&
             run ab_grid2_sm 300 python -u tools/ab_eval.py sm 65536 r5j:8 r5j:2056 r5j:8 r5j:2056 ;;
    abprio3) for c in med lg comp01; do run ab_prio3_$c 400 python -u tools/ab_eval.py $c 65536 r5j:8 q1:8 q2:8 q4:8 r5j:8 q1:8 q2:8 q4:8; done ;;
    lstail) prof_fresh; for c in comp15 comp10 comp01; do run ls_tail_$c 300 python -u tools/ls_tail.py --config $c --dump "$OUT/ls_tail_$c.npz"; done ;;
    abcb) run ab_cb_syn 400 python -u tools/ab_eval.py syn 262144 base:13 cb:13 base:13 cb:13 &&
          run ab_cb_med 300 python -u tools/ab_eval.py med 65536 base:8 cb:8 base:8 cb:8 ;;
    ablp) run ab_lp_syn 400 python -u tools/ab_eval.py syn 262144 r5k:13 lp:13 r5k:13 lp:13 ;;
    gaabx) for i in 1 2; do for c in ${GACFGS:-comp15 comp10 comp01}; do for l in $LIBS; do run ga8k_${c}_${l}_$i 300 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --lib ab_libs/libttga_$l.so; done; done; done ;;
    ablsx) for c in ${LSCFGS:-comp01:8192 med:4096 med:65536 lg:8192}; do run ab_ls_${c%%:*}_${c##*:} 400 python -u tools/ab_ls.py ${c%%:*} ${c##*:} $LIBS; done ;;
    gaisl) for c in ${GACFGS:-comp15 comp10 comp01}; do for k in ${ISLS:-1 2}; do run ga8k_${c}_isl$k 400 python -u tools/bench_ga.py --config $c --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 25 --min-seconds 1.0 --cpu-sample 0 --islands $k; done; done ;;
    isltests) run pytest_isl 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "islands" ;;
    occprobe) run occ_probe 120 tools/occ_probe ;;
    gaisltrace) for k in 1 2; do run ga8k_trace15_isl$k 400 rocprofv3 --kernel-trace --stats -d "$OUT/ga_trace15_isl$k" -o run --output-format csv -- python -u tools/bench_ga.py --config comp15 --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 20 --cpu-sample 0 --islands $k; done ;;
    occsweep) run occ_sweep 120 tools/occ_probe sweep ;;
    t6abl) run t6_ablate 300 python -u tools/eval_variants.py med 65536 8,24,40,9,25,41 ;;
    gacomps20) run ga_comps 900 python -u tools/ga_comps.py "$OUT/ga_comps.json" ;;
    gacomps20i2) run ga_comps_isl2 900 python -u tools/ga_comps.py "$OUT/ga_comps_isl2.json" --islands 2 ;;
    gatrace15) run ga8k_trace15 400 rocprofv3 --kernel-trace --stats -d "$OUT/ga_trace15" -o run --output-format csv -- python -u tools/bench_ga.py --config comp15 --pop 65536 --children 8192 --steps 1000 --warm-gens 96 --warm-feasible 0.6 --gens 20 --cpu-sample 0 ;;
    selftest) run bench_self2 300 env TTGA_BENCH_BACKEND=gloo python -u bench.py --gpus 2 --steps 20 --warmup 2 --no-pmc --no-cpu ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python -u bench.py --no-pmc --no-cpu --steps 100 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "done"
