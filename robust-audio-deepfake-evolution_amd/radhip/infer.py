"""Scoring pass: produce_evaluation_file (src/main.py:958-995) and its data-parallel form.

Score = logits[:, 1] (or the OC-softmax cosine when the criterion carries a `center`). The output is
one line "utt src key score" per trial, in protocol order. The score is written as Python's str() of
the float32 value widened to a double, exactly as the reference's `.tolist()` + "{}".format does.

`produce_evaluation_file_2021` fills the reference's missing 2021-DF scorer (src/main.py:36 comments
out its import; :368 and :761 call it): one "utt score" line per trial of the 2021 protocol, which
`calculate_EER_2021` / the codec report read back (first and last column).

`produce_evaluation_file_sharded` is the multi-GPU eval of SURVEY.md §8e. Each rank scores a
contiguous shard of the trial list; the fp32 scores are all-gathered; rank 0 writes the file in
protocol order. The bytes match the single-process file, because the scores are per-utterance and
the order is fixed by the protocol.
"""
import contextlib

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F


def _scores(model, batch_x, criterion=None, amp=None):
    """amp: None (fp32, the reference's eval), "x3" (fp32 eval with the WavLM stream on the split-precision kernels,
    radhip/wavlm_x3.py) or a dtype to autocast the forward to (bf16 / fp16: the fused 16-bit HIP path)."""
    if amp == "x3":
        from . import wavlm_x3
        ctx = wavlm_x3.scoring()
    elif amp is not None and batch_x.is_cuda:
        ctx = torch.autocast("cuda", dtype=amp)
    else:
        ctx = contextlib.nullcontext()
    with ctx:
        feats, out = model(batch_x)
    feats, out = feats.float(), out.float()
    if criterion is not None and hasattr(criterion, "center"):
        w = F.normalize(criterion.center, p=2, dim=1)
        return F.normalize(feats, p=2, dim=1).mm(w.t()).view(-1)
    return out[:, 1]


def _write(save_path, trial_lines, fnames, scores):
    if not (len(trial_lines) == len(fnames) == len(scores)):
        raise AssertionError(f"{len(trial_lines)} trials, {len(fnames)} utterances, {len(scores)} scores")
    with open(save_path, "w") as fh:
        for fn, sco, trl in zip(fnames, scores, trial_lines):
            _, utt_id, _, src, key = trl.strip().split(" ")
            if fn != utt_id:
                raise AssertionError(f"score order mismatch: {fn} != {utt_id}")
            fh.write("{} {} {} {}\n".format(utt_id, src, key, sco))


def _write_2021(save_path, fnames, scores):
    if len(fnames) != len(scores):
        raise AssertionError(f"{len(fnames)} utterances, {len(scores)} scores")
    with open(save_path, "w") as fh:
        for fn, sco in zip(fnames, scores):
            fh.write("{} {}\n".format(fn, sco))


@torch.no_grad()
def produce_evaluation_file_2021(data_loader, model, device, save_path, criterion=None):
    """data_loader yields (batch_x, utt_ids) in 2021-protocol order; writes "utt score" lines."""
    model.eval()
    fnames, scores = [], []
    for batch_x, utt_id in data_loader:
        s = _scores(model, batch_x.to(device), criterion)
        fnames.extend(utt_id)
        scores.extend(s.float().cpu().numpy().ravel().tolist())
    _write_2021(save_path, fnames, scores)
    print("Scores saved to {}".format(save_path))


@torch.no_grad()
def produce_evaluation_file(data_loader, model, device, save_path, trial_path, criterion=None):
    """data_loader yields (batch_x [B, 64600], utt_ids); writes the score file."""
    model.eval()
    with open(trial_path) as f:
        trial_lines = f.readlines()
    fnames, scores = [], []
    for batch_x, utt_id in data_loader:
        s = _scores(model, batch_x.to(device), criterion)
        fnames.extend(utt_id)
        scores.extend(s.float().cpu().numpy().ravel().tolist())
    _write(save_path, trial_lines, fnames, scores)
    print("Scores saved to {}".format(save_path))


def shard_bounds(n, world, rank):
    """Contiguous shard [lo, hi) of n trials for `rank` (sizes differ by at most one)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _item_batches(dataset, batch_size):
    def gen(lo, hi, device):
        for b0 in range(lo, hi, batch_size):
            items = [dataset[i] for i in range(b0, min(hi, b0 + batch_size))]
            yield torch.stack([torch.as_tensor(it[0]) for it in items]).to(device), [it[1] for it in items]
    return gen


@torch.no_grad()
def produce_evaluation_file_sharded(dataset, model, device, save_path, trial_path, batch_size=32,
                                    criterion=None, group=None, batches=None, fmt="2019", amp=None):
    """dataset[i] -> (x [64600], utt_id) in protocol order. Every rank calls this; rank 0 writes.
    `batches(lo, hi, device)` (e.g. data.EvalFeeder.batches: native decode + GPU pad) replaces the
    item-wise path when given. fmt "2019": "utt src key score" checked against the 5-column trial
    list; fmt "2021": "utt score" in 2021-protocol order."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    model.eval()
    n = len(dataset)
    lo, hi = shard_bounds(n, world, rank)
    batches = batches or _item_batches(dataset, batch_size)
    local = []
    for xb, _ in batches(lo, hi, device):
        local.append(_scores(model, xb, criterion, amp).float())
    local = torch.cat(local) if local else torch.zeros(0, device=device)
    if world > 1:
        width = shard_bounds(n, world, 0)[1]
        buf = torch.zeros(width, device=local.device, dtype=torch.float32)
        buf[:local.numel()] = local
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        scores = torch.cat([p[:shard_bounds(n, world, r)[1] - shard_bounds(n, world, r)[0]]
                            for r, p in enumerate(parts)])
    else:
        scores = local
    if rank == 0:
        fnames = [dataset.utt_id(i) if hasattr(dataset, "utt_id") else dataset[i][1] for i in range(n)]
        vals = scores.cpu().numpy().astype(np.float32).tolist()
        if fmt == "2021":
            _write_2021(save_path, fnames, vals)
        else:
            with open(trial_path) as f:
                trial_lines = f.readlines()
            _write(save_path, trial_lines, fnames, vals)
        print("Scores saved to {}".format(save_path))
    if world > 1:
        dist.barrier(group)
