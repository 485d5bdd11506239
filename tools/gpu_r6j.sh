#!/bin/bash
# LDS operand reads ahead of their MFMAs in sconv_wgrad, the b0x forward / backward and posconv2: their GPU tests
# (sconv, b0x, fixtures, kernels incl. posconv, fp16), micro-benchmarks against the previous build (tools/ab/old:
# HEAD's sconv.hip, b0fused.hip, posconv.hip), then an in-step A/B (new vs old library), two rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6j}
mkdir -p $O
OLD="RADHIP_LIB=$PWD/tools/ab/old/libradhip.so RADHIP_LIB16=$PWD/tools/ab/old/libradhip_f16.so"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sconv_gpu.py tests/test_b0x_gpu.py tests/test_fixtures_gpu.py tests/test_kernels_gpu.py tests/test_f16_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in new old; do
  E=""; [ $v = old ] && E="$OLD"
  env $E timeout -k 10 300 python -u tools/bench_sconv.py --batch 8 32 > $O/sconv_$v.jsonl 2> $O/sconv_$v.err || { tail -5 $O/sconv_$v.err; exit 1; }
  env $E timeout -k 10 300 python -u tools/bench_b0x.py --B 32 --reps 5 --only fused > $O/b0x_$v.txt 2> $O/b0x_$v.err || { tail -5 $O/b0x_$v.err; exit 1; }
  echo "$v b0x: $(tail -3 $O/b0x_$v.txt | tr '\n' ' ')"
  python3 -c "import json; d=[json.loads(l) for l in open('$O/sconv_$v.jsonl') if l.startswith('{')][-1]; print('$v sconv', d)"
done
for r in 1 2; do
  for v in new old; do
    E=""; [ $v = old ] && E="$OLD"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
