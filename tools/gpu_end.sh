# End-of-round evidence: PMC HBM traffic passes (tools/gpu_prof.sh, no trace), then the default bench with the
# bounded CPU baseline. Outputs under gpurun_out/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-end}
mkdir -p gpurun_out/$TAG
NOTRACE=1 TAG=$TAG bash tools/gpu_prof.sh || exit $?
cd $GRAFT_REPO_ROOT
python tools/pmc_traffic.py gpurun_out/$TAG > gpurun_out/$TAG/pmc_traffic.json || exit $?
cp gpurun_out/$TAG/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/$TAG/bench.json'));print('BENCH', d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:400], json.dumps(d['cpu_baseline'])[:300])"
