# In-step A/B of the WavLM GEMM policy: the current radhip.ops.WGEMM_POLICY against the JSON in $OLD (default: the
# round-4 table), two rounds each, bench.py 10 steps, same box.
set -o pipefail
OLD=${OLD:-'{"b8": {"qkv": ["pg", 4, 4], "out": [5, 1], "d_out": [5, 1], "ffn1": [6, 1]}, "b32": {}}'}
TAG=${TAG:-ab}
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_new_$i.json 2> gpurun_out/${TAG}_new_$i.err || exit 1
  RADHIP_WGEMM_POLICY="$OLD" timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_old_$i.json 2> gpurun_out/${TAG}_old_$i.err || exit 1
done
