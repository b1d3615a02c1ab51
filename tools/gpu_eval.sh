set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ev1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "eval" --timeout 120 --timeout-method thread > gpurun_out/ev1/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/ev1/pytest.log
[ $rc -ge 124 ] && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/eval_variants.py med 65536 3,8,9,10,7 > gpurun_out/ev1/variants.json 2>gpurun_out/ev1/err.log
rc=$?; cat gpurun_out/ev1/variants.json; exit $rc
