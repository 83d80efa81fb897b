# The driver's bench command (without the extra legs) alternating between the previous commit's tree (ab_old/) and
# this tree, on one box. Output under gpurun_out/r06ab_bench/.
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r06ab_bench; mkdir -p $OUT
for rep in 1 2 3; do
  for t in ab_old .; do
    timeout -k 10 200 python $t/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/${t//\//_}_$rep.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/${t//\//_}_$rep.log').read().strip().splitlines()[-1]); print('$t', $rep, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
