# hgemm XCD-grid tile order (group_m = -R) against the current policy's column-panel order, in-step, R from $R
# (default 2), every WavLM GEMM shape at both pass sizes; GEMM tests first.
set -o pipefail
R=${R:-2}
TAG=${TAG:-grid}
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -q -k hgemm --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
OLD=$(python3 - <<PY
import json, sys
sys.path.insert(0, "robust-audio-deepfake-evolution_amd")
from radhip.ops import WGEMM_POLICY
print(json.dumps({b: {k: [v[0], v[1], v[2], -$R] for k, v in t.items()} for b, t in WGEMM_POLICY.items()}))
PY
)
echo "$OLD"
TAG=$TAG OLD="$OLD" bash tools/ab_policy.sh
