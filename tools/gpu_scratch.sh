set -u
export TMPDIR=/tmp
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 200 python -u tools/eval_variants.py med 65536 8,1032,7,1031 > $O/med.json 2>$O/err.log || exit $?
cat $O/med.json
timeout -k 10 200 python -u tools/eval_variants.py lg 65536 8,1032 > $O/lg.json 2>>$O/err.log || exit $?
cat $O/lg.json
