set -u
export TMPDIR=/tmp
O=gpurun_out/r02i; mkdir -p $O
# 13 base, 525 prefetch lanes, 1037 w8 corr, 1549 both (13|(32|64)<<4), no-corr 77/589
timeout -k 10 300 python -u tools/eval_variants.py syn 262144 13,525,1037,1549,77,589 > $O/syn.json 2>$O/err.log || exit $?
cat $O/syn.json
