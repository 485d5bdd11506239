# Per-kernel comparison of environment settings: one rocprofv3 kernel trace of a short bench run per setting in
# $SETTINGS (space-separated; "-" = no change; VAR=VALUE[,VAR=VALUE]). Outputs gpurun_out/${TAG}_<i>.csv.gz;
# tools/ab_prof_read.py compares the kernels named on its command line.
set -o pipefail
TAG=${TAG:-abp}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for s in $SETTINGS; do
  envs=""
  [ "$s" != "-" ] && envs=$(echo "$s" | tr ',' ' ')
  for kv in $envs; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/${TAG}_$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/${TAG}_$i.json 2> $O/${TAG}_$i.err || exit 1
  for kv in $envs; do unset "${kv%%=*}"; done
  find /tmp/${TAG}_$i -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$O/${TAG}_$i'.csv.gz' _ {} \;
  echo "setting $i ($s) done"
  i=$((i+1))
done
