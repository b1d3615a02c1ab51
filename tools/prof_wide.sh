set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pw
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pw/prof -o run --output-format csv -- python -u tools/eval_variants.py syn 65536 13 > gpurun_out/pw/log.txt 2>&1; rc=$?
tail -2 gpurun_out/pw/log.txt; exit $rc
