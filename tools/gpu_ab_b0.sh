# A/B of the SincNet block-0 backward kernel (radhip.ops.Block0Convs) against MIOpen's convolutions:
# two default bench runs, RADHIP_FUSED_B0=1 then 0.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/ab/b0_on.json 2> gpurun_out/ab/b0_on.err || exit $?
python3 tools/brief.py gpurun_out/ab/b0_on.json | head -6
RADHIP_FUSED_B0=0 timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/ab/b0_off.json 2> gpurun_out/ab/b0_off.err || exit $?
python3 tools/brief.py gpurun_out/ab/b0_off.json | head -6
