# Tests (env TESTS) then rounds of benches over $VARIANTS lines ("name ENV=VAL ..."; name "base" with no env is
# the default), ROUNDS rounds interleaved; results gpurun_out/$TAG/<name><round>.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-abn}
[ -n "$VARIANTS_FILE" ] && VARIANTS=$(cat $VARIANTS_FILE)
mkdir -p gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest ${TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1; rc=$?
  tail -3 gpurun_out/$TAG/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  printf '%b\n' "$VARIANTS" | while read name envs; do
    [ -z "$name" ] && continue
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/$name$i.json 2> gpurun_out/$TAG/$name$i.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/$TAG/$name$i.json'));print('$name', $i, d['value'])"
  done || exit $?
done
