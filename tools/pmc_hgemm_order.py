"""HBM fetch of csrc/hgemm.hip per launch under its tile orders, for rocprofv3 --pmc FETCH_SIZE: per shape and
group_m value, 3 warm-up + 20 measured launches back to back (operands rotated over 6 copies, as in the 24-layer
pass); the counter CSV lists the dispatches in this order (tools/pmc_hgemm_order_read.py pairs them up).

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o run -- python3 tools/pmc_hgemm_order.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"))
import torch  # noqa: E402

from radhip import ops  # noqa: E402

# (name, M, N, K, tile, splits)
SHAPES = [("b8_ffn2", 1608, 1024, 4096, 4, 2), ("b8_ffn1", 1608, 4096, 1024, 202, 1), ("b8_out", 1608, 1024, 1024, 4, 1),
          ("b32_ffn1", 6432, 4096, 1024, 0, 1), ("b32_ffn2", 6432, 1024, 4096, 2, 1)]
ORDERS = [0, -2, -4, 4]


def main():
    torch.manual_seed(0)
    plan = []
    for name, M, N, K, tile, splits in SHAPES:
        sets = [((torch.randn(M, K, device="cuda") * 0.1).half(), (torch.randn(N, K, device="cuda") * 0.03).half())
                for _ in range(6)]
        for gm in ORDERS:
            for i in range(23):
                a, b = sets[i % 6]
                ops.hgemm(a, b, tile=tile, splits=splits, group_m=gm)
            torch.cuda.synchronize()
            plan.append({"shape": name, "M": M, "N": N, "K": K, "tile": tile, "splits": splits, "group_m": gm,
                         "launches": 23, "warmup": 3,
                         "alg_read_bytes": 2 * (M * K + N * K), "alg_write_bytes": 2 * M * N})
    print(json.dumps(plan))


if __name__ == "__main__":
    main()
