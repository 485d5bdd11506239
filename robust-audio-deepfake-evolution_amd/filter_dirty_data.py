"""Dirty-data filter CLI, drop-in for the reference's src/filter_dirty_data.py (same flags and outputs).

  python filter_dirty_data.py --config config/Phase5_Finetune.conf \
      --model_path exp_result/LA_Phase5_Finetune_ep20_bs12/weights/best.pth \
      --output_path dirty_samples_phase5.txt --filter_ratio 0.02 --batch_size 8 --device cuda --amp
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 filter_dirty_data.py ...

Writes output_path ("utt loss label" for the top filter_ratio of per-utterance CE losses) and the cleaned
protocol output_path.replace(".txt", "_cleaned_protocol.txt"), which Phase6_Run.conf's
data_config.custom_train_protocol points at (src/run_phase6_pipeline.sh:44-70). The work is in
radhip/dirty.py; --device cpu / --allow_cpu are accepted for flag compatibility but this path runs on the
GPU only. Extra: --seed seeds numpy's RNG (pad_random's crops; the reference leaves it unseeded).
"""
import argparse
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from radhip.build import apply_lora_to_wavlm, get_model, load_config, load_weights  # noqa: E402
from radhip.dirty import filter_dirty  # noqa: E402


def main(args):
    config = load_config(args.config)
    if args.device == "cpu" or not torch.cuda.is_available():
        raise RuntimeError("filter_dirty_data runs the MI355X HIP path and needs a ROCm GPU (there is no CPU path)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=device)
    if args.seed is not None:
        np.random.seed(args.seed)
    model = get_model(config["model_config"], device)
    model = apply_lora_to_wavlm(model, config.get("training_config", {}))
    if not os.path.exists(args.model_path):
        raise FileNotFoundError(f"Model file not found: {args.model_path}")
    load_weights(model, args.model_path, device, strict=True)
    dirty, clean = filter_dirty(model, config, args.output_path, batch_size=args.batch_size,
                                filter_ratio=args.filter_ratio, device=device,
                                amp=torch.bfloat16 if args.amp else None, threads=args.loader_threads)
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"Top {args.filter_ratio * 100}% dirty samples: {len(dirty)} of {len(dirty) + len(clean)}")
    if world > 1:
        dist.destroy_process_group()
    return dirty, clean


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Filter dirty training samples based on loss.")
    p.add_argument("--config", type=str, required=True, help="Path to model config file")
    p.add_argument("--model_path", type=str, required=True, help="Path to trained model weights")
    p.add_argument("--output_path", type=str, default="dirty_samples.txt", help="Output file for dirty samples")
    p.add_argument("--batch_size", type=int, default=32, help="Batch size for inference")
    p.add_argument("--filter_ratio", type=float, default=0.02, help="Ratio of samples to filter (e.g., 0.02 for 2%%)")
    p.add_argument("--device", type=str, default="auto", choices=["auto", "cuda", "cpu"], help="Device to use")
    p.add_argument("--allow_cpu", action="store_true", help="accepted for compatibility; the path is GPU-only")
    p.add_argument("--amp", action="store_true", help="bf16 autocast during inference")
    p.add_argument("--seed", type=int, default=None, help="seed numpy's RNG (pad_random crops) first")
    p.add_argument("--loader-threads", dest="loader_threads", type=int, default=8)
    return p.parse_args(argv)


if __name__ == "__main__":
    main(parse_args())
