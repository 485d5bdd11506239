# Targeted GPU tests (TESTS, pytest -k KEXPR), optional micro-benchmarks (PRE: a command), then the bench under
# the tree's defaults and under each variant env of VARIANTS (separated by ';'), ROUNDS times, interleaved.
# Lines in gpurun_out/$TAG/v<k>_<i>.json (v0 = defaults).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-abn}
mkdir -p gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-600} python -u -m pytest $TESTS -m gpu -x -q ${KEXPR:+-k "$KEXPR"} --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1; rc=$?
  tail -3 gpurun_out/$TAG/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PRE" ]; then
  timeout -k 10 300 bash -c "$PRE" > gpurun_out/$TAG/pre.log 2>&1; rc=$?
  cat gpurun_out/$TAG/pre.log | grep -v amdgpu.ids
  [ $rc -eq 0 ] || exit $rc
fi
[ -n "$VARIANTS_FILE" ] && VARIANTS=$(cat "$VARIANTS_FILE")   # variants whose values carry quotes (JSON)
IFS=';' read -ra VS <<< "$VARIANTS"
for i in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/v0_$i.json 2> gpurun_out/$TAG/v0_$i.err || exit $?
  k=1
  for v in "${VS[@]}"; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/v${k}_$i.json 2> gpurun_out/$TAG/v${k}_$i.err || exit $?
    k=$((k+1))
  done
  python - "$TAG" "$i" "${#VS[@]}" <<'PY'
import json, sys
tag, i, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
vals = [json.load(open(f"gpurun_out/{tag}/v{k}_{i}.json"))["value"] for k in range(n + 1)]
print("round", i, " ".join(f"v{k}={v}" for k, v in enumerate(vals)))
PY
done
