"""Dirty-data filter (the step that defines the Phase6_Run training set), on the MI355X scoring path.

Reference: src/filter_dirty_data.py:37-206, driven by src/run_phase6_pipeline.sh:14-21 (Phase-5 best.pth,
filter ratio 0.02, batch 8, --amp). Semantics kept:
  * the train protocol (database_path/ASVspoof2019_{track}_cm_protocols/...cm.train.trn.txt, never the
    custom_train_protocol) in file order, labels bonafide = 1;
  * the items of Dataset_ASVspoof2019_train with algo 0 and no codec: pad_random, i.e. for an
    utterance longer than 64 600 samples a crop at np.random.randint(len - 64600) drawn from numpy's
    global RNG in protocol order (the reference does not seed it; --seed does here), tiling otherwise;
  * eval-mode forward, per-utterance CrossEntropyLoss(reduction='none') on the logits (no class
    weights), softmax probability of the true class;
  * Python's stable sort by loss, descending; the first int(N * ratio) are dirty;
  * "{file} {loss:.6f} {label}" lines for the dirty samples; the cleaned protocol is the clean samples'
    original protocol lines in the SORTED order (descending loss), written to output_path with every
    ".txt" replaced by "_cleaned_protocol.txt" (str.replace, as the reference).
Differences: weights load strictly (the reference's strict=False would silently score a mismatched
model); --amp is bf16 autocast; N * ratio < 1 writes an empty dirty list instead of the reference's
IndexError on `dirty_samples[0]`; a 64 600-sample utterance is taken whole (the reference's randint(0)
raises). The decode is native and the crop/tile is the GPU pad kernel; with several ranks the protocol
is scored in contiguous shards and the losses all-gathered (every rank draws the full crop sequence,
so the result does not depend on the world size).
"""
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import audio
from .data import CUT, genSpoof_list
from .infer import shard_bounds
from .ops import pad_mixup


def crop_starts(lens, max_len=CUT):
    """pad_random's crop starts, one numpy draw per utterance longer than max_len, in order."""
    return [int(np.random.randint(n - max_len)) if n > max_len else 0 for n in lens]


def train_batches(paths, starts, lo, hi, batch_size, device, threads=8):
    """[B, 64600] GPU batches of utterances lo..hi-1: native decode, then crop at `starts` or tile."""
    for b0 in range(lo, hi, batch_size):
        idx = list(range(b0, min(hi, b0 + batch_size)))
        flat, offs, lens = audio.read_batch([paths[i] for i in idx], threads=threads)
        dev = torch.from_numpy(flat).to(device, non_blocking=False)
        yield pad_mixup(dev, offs.tolist(), lens.tolist(), [starts[i] for i in idx], CUT)


@torch.no_grad()
def score_losses(model, paths, labels, batch_size, device, amp=None, threads=8, group=None):
    """Per-utterance (CE loss, probability of the true class), float32, in protocol order."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    n = len(paths)
    starts = crop_starts([audio.probe(p)[0] for p in paths])
    lo, hi = shard_bounds(n, world, rank)
    y_all = torch.tensor(labels, dtype=torch.long, device=device)
    model.eval()
    out = []
    b0 = lo
    for xb in train_batches(paths, starts, lo, hi, batch_size, device, threads):
        y = y_all[b0:b0 + xb.shape[0]]
        with torch.autocast("cuda", dtype=amp or torch.bfloat16, enabled=amp is not None):
            _, logits = model(xb, Freq_aug=False)
        logits = logits.float()
        loss = F.cross_entropy(logits, y, reduction="none")
        prob = torch.softmax(logits, dim=1).gather(1, y[:, None])[:, 0]
        out.append(torch.stack([loss, prob], dim=1))
        b0 += xb.shape[0]
    local = torch.cat(out) if out else torch.zeros(0, 2, device=device)
    if world > 1:
        width = shard_bounds(n, world, 0)[1]
        buf = torch.zeros(width, 2, device=device)
        buf[:local.shape[0]] = local
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        local = torch.cat([p[:shard_bounds(n, world, r)[1] - shard_bounds(n, world, r)[0]]
                           for r, p in enumerate(parts)])
    res = local.cpu().numpy().astype(np.float32)
    return res[:, 0], res[:, 1]


def select_dirty(files, losses, labels, probs, ratio):
    """(dirty, clean) record lists: stable sort by loss, descending; the first int(N * ratio) are dirty."""
    results = [{"file": f, "loss": float(l), "label": int(y), "prob": float(p)}
               for f, l, y, p in zip(files, losses, labels, probs)]
    results.sort(key=lambda r: r["loss"], reverse=True)
    k = int(len(results) * ratio)
    return results[:k], results[k:]


def write_outputs(output_path, dirty, clean, protocol_lines):
    """Writes the dirty list and the cleaned protocol; returns the cleaned protocol's path."""
    with open(output_path, "w") as f:
        for r in dirty:
            f.write(f"{r['file']} {r['loss']:.6f} {r['label']}\n")
    clean_path = str(output_path).replace(".txt", "_cleaned_protocol.txt")
    with open(clean_path, "w") as f:
        for r in clean:
            line = protocol_lines.get(r["file"])
            if line is None:
                line = f"LA_0000 {r['file']} - - {'bonafide' if r['label'] == 1 else 'spoof'}"
            f.write(line + "\n")
    return clean_path


def protocol_line_map(path):
    lines = {}
    with open(path) as f:
        for line in f:
            parts = line.strip().split()
            if len(parts) >= 2:
                lines[parts[1]] = line.strip()
    return lines


def train_protocol(config):
    db = Path(config["database_path"])
    track = config["track"]
    return (db / "ASVspoof2019_{}_cm_protocols/ASVspoof2019.{}.cm.train.trn.txt".format(track, track),
            db / f"ASVspoof2019_{track}_train")


def filter_dirty(model, config, output_path, batch_size=32, filter_ratio=0.02, device="cuda", amp=None,
                 threads=8, group=None):
    """The whole filter on a built, loaded model; rank 0 writes. Returns (dirty, clean) records."""
    trn, base = train_protocol(config)
    proto = protocol_line_map(trn)
    labels, files = genSpoof_list(trn, is_train=True, is_eval=False)
    paths = [base / f"flac/{k}.flac" for k in files]
    ys = [labels[k] for k in files]
    losses, probs = score_losses(model, paths, ys, batch_size, device, amp, threads, group)
    dirty, clean = select_dirty(files, losses, ys, probs, filter_ratio)
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1 or dist.get_rank(group) == 0:
        write_outputs(output_path, dirty, clean, proto)
    return dirty, clean
