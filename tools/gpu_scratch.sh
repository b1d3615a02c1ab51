set -u
export TMPDIR=/tmp
O=gpurun_out/r02zo; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u tools/eval_variants.py med 65536 8,7 > $O/med.json 2>>$O/err.log || exit $?
timeout -k 10 200 python -u tools/eval_variants.py lg 65536 8,7 > $O/lg.json 2>>$O/err.log || exit $?
timeout -k 10 300 python -u tools/eval_variants.py syn 262144 13 > $O/syn.json 2>>$O/err.log || exit $?
cat $O/med.json $O/lg.json $O/syn.json
exit $rc
