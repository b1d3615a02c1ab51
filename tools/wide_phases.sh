set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/wph
timeout -k 10 200 python -u tools/eval_variants.py syn 65536 13,29,45,61 > gpurun_out/wph/phases.json 2>gpurun_out/wph/err.log; rc=$?
cat gpurun_out/wph/phases.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/eval_variants.py med 65536 8,9,13 > gpurun_out/wph/med.json 2>>gpurun_out/wph/err.log; rc=$?
cat gpurun_out/wph/med.json; exit $rc
