# kernel + fused tests, attention sweep, then the bench (stops at the first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/it
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_wavlm_fused_gpu.py} -x -v --timeout 300 --timeout-method thread > gpurun_out/it/pytest.log 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" gpurun_out/it/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/it/sweep.jsonl
for ns in ${SWEEP:-2,2,4 4,4,4}; do
  RADHIP_ATTN_NS=$ns timeout -k 10 120 python tools/bench_attn.py >> gpurun_out/it/sweep.jsonl 2>> gpurun_out/it/err.log || exit 1
done
cat gpurun_out/it/sweep.jsonl
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/it/bench.json 2> gpurun_out/it/bench.err; rc=$?
python3 -c "import json;d=json.load(open('gpurun_out/it/bench.json'));print('VALUE',d['value'],'ms/step',d['ms_per_step'],'loss',d['final_loss']);print({k:(round(v['avg_ms']*1e3,1),v['launches']) for k,v in d['kernels'].items()})"
exit $rc
