#!/bin/bash
# sconv_wgrad (64 x 64 channels only) with its MFMA operand reads two steps ahead: sconv / fixture tests, the
# per-shape micro-benchmark in alternating order against the previous build (tools/ab/old), then an in-step A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6r}
mkdir -p $O
OLD="RADHIP_LIB=$PWD/tools/ab/old/libradhip.so RADHIP_LIB16=$PWD/tools/ab/old/libradhip_f16.so"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sconv_gpu.py tests/test_fixtures_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
i=0
for v in old new old new; do
  i=$((i+1)); E=""; [ $v = old ] && E="$OLD"
  env $E timeout -k 10 300 python -u tools/bench_sconv.py --batch 8 32 > $O/sconv_${v}_$i.jsonl 2> $O/sconv_${v}_$i.err || { tail -5 $O/sconv_${v}_$i.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/sconv_${v}_$i.jsonl') if l.startswith('{')]; print('$v', [(r['B'], r['conv'], round(r['sconv_fwdbwd_us']-r['sconv_fwd_us'],1)) for r in d if 'B' in r and r['conv'] in ('b2.conv2','b3.conv1','b3.conv2','b1.conv2')])"
done
for r in 1 2; do
  for v in old new; do
    E=""; [ $v = old ] && E="$OLD"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
