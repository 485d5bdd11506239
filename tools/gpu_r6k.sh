#!/bin/bash
# b0x backward and posconv2 with their LDS operand reads ahead of the MFMAs (sconv_wgrad and the b0x forward
# variants of r6j reverted): tests, micro-benchmarks new vs old (tools/ab/old = the round's previous commit), in-step
# A/B with the order of the variants alternated.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6k}
mkdir -p $O
OLD="RADHIP_LIB=$PWD/tools/ab/old/libradhip.so RADHIP_LIB16=$PWD/tools/ab/old/libradhip_f16.so"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sconv_gpu.py tests/test_b0x_gpu.py tests/test_fixtures_gpu.py tests/test_kernels_gpu.py tests/test_f16_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in old new old new; do
  E=""; [ $v = old ] && E="$OLD"
  env $E timeout -k 10 300 python -u tools/bench_b0x.py --B 32 --reps 5 --only fused > $O/b0x_$v.txt 2> $O/b0x_$v.err || { tail -5 $O/b0x_$v.err; exit 1; }
  env $E timeout -k 10 300 python -u tools/bench_kernels.py > $O/kern_$v.txt 2> $O/kern_$v.err || { tail -5 $O/kern_$v.err; exit 1; }
  echo "$v b0x: $(tail -1 $O/b0x_$v.txt) posconv: $(grep -o '"posconv[a-z_]*": [0-9.]*' $O/kern_$v.txt | tr '\n' ' ')"
done
for r in 1 2; do
  for v in old new; do
    E=""; [ $v = old ] && E="$OLD"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
