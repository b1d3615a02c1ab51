# eval_tile5 (variant 8) ablations, profiling only: 1 lane phase, 2 wave phase, 4 corr words,
# 8 B-bitset atomics, 16 cell-counter atomics, 32 workspace zeroing (ablated results are invalid)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/t5ph
timeout -k 10 200 python -u tools/eval_variants.py med 65536 8,24,40,72,136,264,520,392,920 > gpurun_out/t5ph/phases.json 2>gpurun_out/t5ph/err.log; rc=$?
cat gpurun_out/t5ph/phases.json; exit $rc
