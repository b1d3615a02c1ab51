set -u
export TMPDIR=/tmp
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 500 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 8192 --steps 1000 --warm-gens 400 --warm-feasible 0.6 --gens 10 --cpu-sample 64 > $O/ga_p2_c8k.json 2>$O/err.log || exit $?
cat $O/ga_p2_c8k.json
timeout -k 10 500 python -u tools/bench_ga.py --config comp01 --pop 65536 --children 32768 --steps 1000 --warm-gens 400 --warm-feasible 0.6 --gens 5 --cpu-sample 0 > $O/ga_p2_c32k.json 2>>$O/err.log || exit $?
cat $O/ga_p2_c32k.json
