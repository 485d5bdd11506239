# In-step comparison of several environment settings on one box: bench.py (10 steps, no CPU leg) once per
# setting in $SETTINGS (space-separated; "-" = no change; a setting is VAR=VALUE[,VAR=VALUE]), two rounds.
# Outputs gpurun_out/${TAG}_<i>_<round>.json.
set -o pipefail
TAG=${TAG:-abm}
for r in 1 2; do
  i=0
  for s in $SETTINGS; do
    envs=""
    [ "$s" != "-" ] && envs=$(echo "$s" | tr ',' ' ')
    env $envs timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_${i}_$r.json 2> gpurun_out/${TAG}_${i}_$r.err || exit 1
    i=$((i+1))
  done
done
