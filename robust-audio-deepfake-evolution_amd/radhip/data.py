"""ASVspoof data path: protocol parsing, padding, datasets and the GPU micro-batch feeder.

Reference: src/data_utils.py
  genSpoof_list :62-104        -> gen_spoof_list / genSpoof_list (same return structure, bit-exact order)
  pad :107-114, pad_random :117-127
  Dataset_ASVspoof2019_train :130-184, Dataset_ASVspoof2019_devNeval :187-203,
  Dataset_ASVspoof2021_eval :206-229, Dataset_InTheWild :233-271
  get_loader (src/main.py:815-955): train order = torch.randperm(n, generator=Generator(seed)) per epoch
  (DataLoader(shuffle=True, generator=gen, drop_last=True)), dev/eval in protocol order.

MI355X design: the datasets keep the reference's per-item API (x, key/label) for parity and tools, but
the train/eval drivers do not go through them item by item. `TrainFeeder` decodes a whole micro-batch
with the native multi-threaded FLAC loader into a pinned buffer, makes the per-utterance augmentation
draws on the host in the reference's RNG order, and runs RawBoost / codec resampling / pad_random /
mixup as batched HIP kernels (radhip.train.Augmenter). `EvalFeeder` does the same with the eval pad.
"""
from pathlib import Path

import numpy as np
import torch

from . import audio

CUT = 64600  # ~4 s at 16 kHz (data_utils.py:137)


def str_to_bool(val):
    """distutils.strtobool semantics (src/utils.py:13-31)."""
    v = str(val).lower()
    if v in ("y", "yes", "t", "true", "on", "1"):
        return True
    if v in ("n", "no", "f", "false", "off", "0"):
        return False
    raise ValueError(f"invalid truth value {val!r}")


def genSpoof_list(dir_meta, is_train=False, is_eval=False, is_2021=False):
    """Protocol parse with the reference's return structure: 2021 -> [keys]; eval -> [keys];
    train/dev -> ({key: 1 bonafide / 0 spoof}, [keys]). Lines are split on single spaces like the
    reference (a malformed line raises ValueError there and here)."""
    with open(dir_meta, "r") as f:
        lines = f.readlines()
    if is_2021:
        keys = []
        for line in lines:
            line = line.strip()
            if not line:
                continue
            parts = line.split()
            keys.append(parts[1] if len(parts) >= 2 else parts[0])
        return keys
    labels, keys = {}, []
    for line in lines:
        _, key, _, _, label = line.strip().split(" ")
        keys.append(key)
        if is_train or not is_eval:
            labels[key] = 1 if label == "bonafide" else 0
    if is_eval and not is_train:
        return keys
    return labels, keys


def pad(x, max_len=CUT):
    """Eval pad: head crop, or tile (data_utils.py:107-114)."""
    n = x.shape[0]
    if n >= max_len:
        return x[:max_len]
    reps = int(max_len / n) + 1
    return np.tile(x, (1, reps))[:, :max_len][0]


def pad_random(x, max_len=CUT):
    """Train pad: random crop at np.random.randint(len - max_len), or tile (data_utils.py:117-127).
    Like the reference, a length of exactly max_len raises (randint(0))."""
    n = x.shape[0]
    if n >= max_len:
        stt = np.random.randint(n - max_len)
        return x[stt:stt + max_len]
    reps = int(max_len / n) + 1
    return np.tile(x, reps)[:max_len]


class Dataset_ASVspoof2019_devNeval(torch.utils.data.Dataset):
    """(x [64600] fp32, key) in protocol order (data_utils.py:187-203)."""

    def __init__(self, list_IDs, base_dir):
        self.list_IDs, self.base_dir, self.cut = list_IDs, Path(base_dir), CUT

    def __len__(self):
        return len(self.list_IDs)

    def path(self, i):
        return self.base_dir / f"flac/{self.list_IDs[i]}.flac"

    def utt_id(self, i):
        return self.list_IDs[i]

    def __getitem__(self, index):
        X, _ = audio.read(self.path(index))
        return torch.tensor(pad(X, self.cut), dtype=torch.float32), self.list_IDs[index]


class Dataset_ASVspoof2021_eval(Dataset_ASVspoof2019_devNeval):
    """2021 DF eval (data_utils.py:206-229): an unreadable file becomes zeros, with a warning."""

    def __getitem__(self, index):
        key = self.list_IDs[index]
        try:
            X, _ = audio.read(self.path(index))
        except (audio.AudioReadError, OSError) as e:
            print(f"Warning: Failed to read {key}.flac: {e}. Using zero-padded audio.")
            X = np.zeros(self.cut, dtype=np.float32)
        return torch.tensor(pad(X, self.cut), dtype=torch.float32), key


class Dataset_ASVspoof2019_train(torch.utils.data.Dataset):
    """Per-item train dataset with the reference's CPU augmentation order (data_utils.py:130-184).
    The GPU train path uses TrainFeeder instead; this exists for API parity (item-level tools)."""

    def __init__(self, list_IDs, labels, base_dir, algo=0, use_codec=False, codec_p=0.5, rawboost_p=1.0):
        self.list_IDs, self.labels, self.base_dir = list_IDs, labels, Path(base_dir)
        self.cut, self.algo, self.use_codec = CUT, algo, use_codec
        self.codec_p, self.rawboost_p = float(codec_p), float(rawboost_p)

    def __len__(self):
        return len(self.list_IDs)

    def path(self, i):
        return self.base_dir / f"flac/{self.list_IDs[i]}.flac"

    def __getitem__(self, index):
        """One augmented item (x [64600] fp32 on the host, label), the reference's draw order, with
        RawBoost/codec/pad_random on the GPU augmenter (there is no CPU augmentation path)."""
        if getattr(self, "_aug", None) is None:
            from .train import Augmenter
            self._aug = Augmenter("cuda", self.algo, self.rawboost_p, self.use_codec, self.codec_p, self.cut)
        key = self.list_IDs[index]
        X, _ = audio.read(self.path(index))
        raw = torch.tensor(X, dtype=torch.float32, device=self._aug.device)
        plan = self._aug.draw([raw.numel()])
        x = self._aug.run(raw, [0], [raw.numel()], plan)
        return x[0].cpu(), self.labels[key]


class Dataset_InTheWild(torch.utils.data.Dataset):
    """meta.csv (file, label) + wav files (data_utils.py:233-271); label 0 bona-fide, 1 spoof."""

    def __init__(self, meta_csv, base_dir, sample_rate=16000):
        import csv
        self.base_dir, self.cut, self.sample_rate = Path(base_dir), CUT, sample_rate
        with open(meta_csv, newline="") as f:
            rows = list(csv.DictReader(f))
        if not rows or not {"file", "label"}.issubset(rows[0].keys()):
            raise ValueError("meta.csv must have columns file, label")
        self.files = [r["file"] for r in rows]
        self.labels = [r["label"] for r in rows]

    def __len__(self):
        return len(self.files)

    def __getitem__(self, index):
        fname = self.files[index]
        label = 0 if self.labels[index].lower() == "bona-fide" else 1
        try:
            X, sr = audio.read(self.base_dir / fname)
            if sr != self.sample_rate:
                raise audio.AudioReadError(f"{fname}: sample rate {sr} != {self.sample_rate}")
        except (audio.AudioReadError, OSError) as e:
            print(f"Warning: Failed to read {fname}: {e}. Using zero-padded audio.")
            X = np.zeros(self.cut, dtype=np.float32)
        return torch.tensor(pad(X, self.cut), dtype=torch.float32), label, fname


# ------------------------------------------------------------------ GPU feeders -------------
class _PinnedBuf:
    """Pinned staging buffer; get() waits for the previous non_blocking H2D copy out of it."""

    def __init__(self):
        self.t = None
        self.ev = None

    def get(self, n):
        if self.ev is not None:
            self.ev.synchronize()
            self.ev = None
        if self.t is None or self.t.numel() < n:
            self.t = torch.empty(max(n, 1 << 20), dtype=torch.float32, pin_memory=torch.cuda.is_available())
        return self.t

    def upload(self, n, device):
        dev = self.t[:n].to(device, non_blocking=True)
        if dev.is_cuda:
            self.ev = torch.cuda.Event()
            self.ev.record()
        return dev


class TrainFeeder:
    """Shuffled micro-batches of the train list (drop_last=True), augmented on the GPU.

    Order: what the reference's DataLoader(shuffle=True, drop_last=True, generator=gen) draws from
    gen = Generator().manual_seed(seed) (main.py:909-920) on torch 2.x, per epoch: the iterator's base
    seed (one int64 random_), RandomSampler's torch.randperm(n) (the order used), and the sampler's
    trailing randperm(n)[:n % n] that runs when the exhausted sampler is polled once more
    (tests/test_data_cpu.py compares against a real DataLoader over several epochs).
    Per micro-batch: native batch decode -> Augmenter.draw (python/numpy RNG in __getitem__ order) ->
    mixup draw (np.random.beta, torch.randperm) -> Augmenter.run (RawBoost, codec, pad_random, mixup)."""

    def __init__(self, keys, labels, base_dir, batch_size, augmenter, seed, threads=8, rank=0, world=1):
        self.keys, self.labels, self.base_dir = list(keys), labels, Path(base_dir)
        self.B, self.aug, self.threads = int(batch_size), augmenter, threads
        self.gen = torch.Generator()
        self.gen.manual_seed(seed)
        self.rank, self.world = rank, world
        self.pin = _PinnedBuf()

    def __len__(self):
        """Micro-batches per epoch on this rank (global batches = world * B utterances)."""
        return len(self.keys) // (self.B * self.world)

    def epoch_order(self):
        """This epoch's shuffled index order, consuming the generator exactly as one full pass of the
        reference's DataLoader does."""
        n = len(self.keys)
        torch.empty((), dtype=torch.int64).random_(generator=self.gen)    # _BaseDataLoaderIter base seed
        order = torch.randperm(n, generator=self.gen).tolist()              # RandomSampler.__iter__
        torch.randperm(n, generator=self.gen)                               # its trailing [:n % n] draw
        return order

    def epoch(self):
        order = self.epoch_order()
        gb = self.B * self.world
        for i in range(len(self)):
            chunk = order[i * gb:(i + 1) * gb][self.rank * self.B:(self.rank + 1) * self.B]
            yield [self.keys[j] for j in chunk]

    def load(self, keys, device):
        """Decode + upload one micro-batch: returns (flat device buffer, offsets, lens, labels)."""
        paths = [self.base_dir / f"flac/{k}.flac" for k in keys]
        lens = [audio.probe(p)[0] for p in paths]
        host = self.pin.get(int(sum(lens)))
        _, offs, lens = audio.read_batch(paths, out=host, threads=self.threads)
        dev = self.pin.upload(int(lens.sum()), device)
        y = torch.tensor([self.labels[k] for k in keys], dtype=torch.long)
        return dev, offs.tolist(), lens.tolist(), y


class EvalFeeder:
    """Protocol-order eval batches: decode (native) -> GPU pad (head crop / tile) -> [B, 64600]."""

    def __init__(self, dataset, batch_size, threads=8, zero_on_error=False):
        self.ds, self.B, self.threads, self.zero_on_error = dataset, int(batch_size), threads, zero_on_error
        self.pin = _PinnedBuf()

    def batches(self, lo, hi, device):
        from .ops import pad_mixup
        for b0 in range(lo, hi, self.B):
            idx = list(range(b0, min(hi, b0 + self.B)))
            paths = [self.ds.path(i) for i in idx]
            keys = [self.ds.utt_id(i) for i in idx]
            try:
                lens = [audio.probe(p)[0] for p in paths]
                host = self.pin.get(int(sum(lens)))
                _, offs, lens = audio.read_batch(paths, out=host, threads=self.threads)
            except (audio.AudioReadError, OSError):
                if not self.zero_on_error:
                    raise
                yield self._item_batch(idx, device), keys
                continue
            dev = self.pin.upload(int(lens.sum()), device)
            yield pad_mixup(dev, offs.tolist(), lens.tolist(), [0] * len(idx), CUT), keys

    def _item_batch(self, idx, device):
        return torch.stack([self.ds[i][0] for i in idx]).to(device)
