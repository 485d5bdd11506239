# In-step A/B of one environment switch: bench.py (10 steps, no CPU leg) with $ENV_B set vs unset, two rounds each,
# same box. Outputs gpurun_out/${TAG}_{a,b}_{1,2}.json.
set -o pipefail
TAG=${TAG:-abenv}
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_a_$i.json 2> gpurun_out/${TAG}_a_$i.err || exit 1
  env $ENV_B timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_b_$i.json 2> gpurun_out/${TAG}_b_$i.err || exit 1
done
