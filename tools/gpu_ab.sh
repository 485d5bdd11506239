# A/B of bench variants: each line of $VARIANTS is "name ENV=VAL ..." (empty env = default); one bench each,
# no CPU baseline, results under gpurun_out/$TAG/<name>.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-ab}
mkdir -p gpurun_out/$TAG
echo "$VARIANTS" | while read name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/$TAG/$name.json'));print('$name', d['value'], d['ms_per_step'])"
done
