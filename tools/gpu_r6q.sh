#!/bin/bash
# attention cross-half exchanges on permlane32 swaps, the LN1 gate reduction on permlane / DPP:
# backward): their GPU tests and the model / e2e tests, a kernel trace of a short bench run (per-kernel times of the
# head launches), then an in-step A/B against the previous build (tools/ab/old = the round's previous commit).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6l}
mkdir -p $O
OLD="RADHIP_LIB=$PWD/tools/ab/old/libradhip.so RADHIP_LIB16=$PWD/tools/ab/old/libradhip_f16.so"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_wavlm_fused_gpu.py tests/test_f16_gpu.py tests/test_e2e_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
rm -rf /tmp/$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$1 -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err || { tail -10 $O/prof.err; exit 1; }
find /tmp/$1 -name "*kernel_stats.csv" -exec cp {} $O/ \;
grep -E "wl_ln1|attn_fwd|attn_bwd" $O/run_kernel_stats.csv | cut -c1-120 || true
for r in 1 2; do
  for v in old new; do
    E=""; [ $v = old ] && E="$OLD"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
