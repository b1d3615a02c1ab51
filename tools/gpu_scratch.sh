set -u
export TMPDIR=/tmp
O=gpurun_out/r02p; mkdir -p $O
# round-1 long-run workload (pop 4096, 200 generations, maxSteps 1000)
timeout -k 10 300 python -u tools/bench_ga.py --config comp01 --pop 4096 --children 4096 --steps 1000 --gens 200 --cpu-sample 64 > $O/ga_long.json 2>$O/err.log || exit $?
cat $O/ga_long.json
# phase-2 headline: warm until 60% feasible, then 10 timed generations
timeout -k 10 500 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --steps 1000 --warm-gens 400 --warm-feasible 0.6 --gens 10 --cpu-sample 64 > $O/ga_p2.json 2>>$O/err.log || exit $?
cat $O/ga_p2.json
