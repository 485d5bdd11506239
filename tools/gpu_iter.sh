# build -> kernel/model GPU tests -> bench (graphs) ; stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
make -C robust-audio-deepfake-evolution_amd/csrc -j8 > /dev/null || exit 1
timeout -k 10 900 python -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_model_gpu.py} -x -q > gpurun_out/pt.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/pt.log | tail -${TAILN:-4}
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err; rc=$?
grep -v amdgpu.ids gpurun_out/bench_iter.err | tail -3
python3 -c "import json;d=json.load(open('gpurun_out/bench_iter.json'));print('VALUE',d['value'],'ms/step',d['ms_per_step'],'loss',d['final_loss']);print({k:(round(v['avg_ms']*1e3,1),v['launches']) for k,v in d['kernels'].items()})"
exit $rc
