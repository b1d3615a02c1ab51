set -u
export TMPDIR=/tmp
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 200 python -u tools/time_problem.py $O/time_problem.json > $O/time_problem.log 2>&1 || exit $?
tail -4 $O/time_problem.log
timeout -k 10 300 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 128 > $O/ls_p2.json 2>$O/err.log || exit $?
cat $O/ls_p2.json
timeout -k 10 300 python -u tools/ls_prof.py --pop 4096 --steps 1000 --pre-steps 3000 > $O/ls_prof_p2.json 2>>$O/err.log || exit $?
timeout -k 10 400 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 65536 --steps 1000 --warm-gens 80 --warm-feasible 0.6 --gens 3 --cpu-sample 64 > $O/ga_p2.json 2>>$O/err.log || exit $?
cat $O/ga_p2.json
