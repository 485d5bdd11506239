set -o pipefail
OLD='{"b8": {"qkv": ["pg", 4, 4], "out": [5, 1], "d_out": [5, 1], "ffn1": [6, 1]}, "b32": {}}'
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_new_$i.json 2> gpurun_out/ab_new_$i.err || exit 1
  RADHIP_WGEMM_POLICY="$OLD" timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_old_$i.json 2> gpurun_out/ab_old_$i.err || exit 1
done
