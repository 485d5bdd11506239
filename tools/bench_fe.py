"""The frozen WavLM CNN (radhip.ops.feature_encoder_fused) at the window's clean batch (32 x 64600): total time per
tile of the strided-convolution GEMMs (RADHIP_FE_TILE semantics: -1 = csrc/gemm.hip, else an hgemm tile), and the
conv0 kernel alone. One JSON line per case.

    python tools/bench_fe.py [--batch 32]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"), ROOT]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    from radhip import ops
    from radhip.wavlm import FeatureEncoder, WavLMConfigLite
    dev = torch.device("cuda", 0)
    fe = FeatureEncoder(WavLMConfigLite()).to(dev).eval()
    for p in fe.parameters():
        p.requires_grad_(False)
    x = (0.1 * torch.randn(a.batch, 64600, device=dev)).clamp(-1, 1)
    for dt in (torch.float16, torch.bfloat16):
        W = ops.fe_conv_weights(fe.conv_layers, dt)
        for tile in (-1, 0, 2, 4):
            ops.FE_HGEMM_TILE = tile
            for _ in range(3):
                ops.feature_encoder_fused(x, W)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(10):
                ops.feature_encoder_fused(x, W)
            e.record()
            torch.cuda.synchronize()
            print(json.dumps({"dtype": str(dt), "tile": tile, "ms": round(s.elapsed_time(e) / 10, 3)}), flush=True)


if __name__ == "__main__":
    main()
