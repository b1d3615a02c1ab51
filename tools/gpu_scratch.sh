set -u
export TMPDIR=/tmp
O=gpurun_out/r02r; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ga.py tests/test_gpu_configs.py -x -q -k "local_search or ls or ga or island or rng or config" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_ls.py --pop 4096 --steps 1000 --pre-steps 3000 --cpu-sample 128 > $O/ls_p2.json 2>$O/err.log || exit $?
cat $O/ls_p2.json
timeout -k 10 300 python -u tools/bench_ls.py --pop 4096 --steps 200 --cpu-sample 128 > $O/ls_p1.json 2>>$O/err.log || exit $?
cat $O/ls_p1.json
timeout -k 10 300 python -u tools/ls_prof.py --pop 4096 --steps 1000 --pre-steps 3000 > $O/prof_p2.json 2>>$O/err.log || exit $?
timeout -k 10 300 python -u tools/bench_ga.py --config comp01 --pop 4096 --children 4096 --steps 1000 --gens 200 --cpu-sample 0 > $O/ga_long.json 2>>$O/err.log || exit $?
cat $O/ga_long.json
