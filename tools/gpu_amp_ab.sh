# bench.py under bf16 and fp16 autocast back to back (no CPU baseline): gpurun_out/$TAG/{bf16,fp16}.json
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-amp}
O=gpurun_out/$TAG
mkdir -p $O
for a in ${AMPS:-bf16 fp16}; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --amp $a ${BENCH_ARGS} > $O/$a.json 2> $O/$a.err || exit $?
  python -c "import json; d=json.load(open('$O/$a.json')); print('$a', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
