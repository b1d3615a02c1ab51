# Six self-launched two-rank rehearsals of bench.py (gloo, both ranks on the one GPU),
# printing each line's rank verification; stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06_ag
for i in 1 2 3 4 5 6; do
  TTGA_BENCH_BACKEND=gloo timeout -k 10 240 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-pmc --no-cpu > gpurun_out/r06_ag/self2_$i.log 2> gpurun_out/r06_ag/self2_$i.err || { echo "run $i rc=$?"; exit 1; }
  python -c "
import json,sys
l=[x for x in open('gpurun_out/r06_ag/self2_$i.log') if x.startswith('{')][-1]
d=json.loads(l); r=d['ranks']; print($i, r['ranks_verified'], r['world'], [x.get('mismatch') for x in r['devices']])"
done
