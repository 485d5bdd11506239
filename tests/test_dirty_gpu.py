"""Dirty-data filter end to end on the GPU (filter_dirty_data.py -> radhip/dirty.py): the reference's
toy-scorer run (tests/golden/dirty_filter.json) is replayed on FLAC files holding the same samples, with
the same numpy seed for pad_random's crops. The cleaned protocol (what Phase6_Run trains on) must equal the
reference's byte for byte; the dirty list must have the reference's utterances, order and labels, with
losses within fp32 rounding of the GPU's logits."""
import json
import sys
import types

import numpy as np
import pytest
import torch

from flac_writer import encode
from seeded import dirty_audio

pytestmark = pytest.mark.gpu


class ToyScore(torch.nn.Module):
    """The toy scorer of make_golden.gen_dirty: logits [0, w0 * mean(x) + w1]."""

    def __init__(self, args, device):
        super().__init__()
        self.w = torch.nn.Parameter(torch.tensor([40.0, 0.05]))

    def forward(self, x, Freq_aug=False):
        z = self.w[0] * x.mean(dim=1) + self.w[1]
        return x[:, :4], torch.stack([torch.zeros_like(z), z], dim=1)


def test_filter_dirty_data_cli_matches_reference(golden, tmp_path, monkeypatch):
    import filter_dirty_data as fdd
    g = golden("dirty_filter.json")
    mod = types.ModuleType("models.ToyScore")
    mod.Model = ToyScore
    monkeypatch.setitem(sys.modules, "models.ToyScore", mod)
    db = tmp_path / "LA"
    (db / "ASVspoof2019_LA_cm_protocols").mkdir(parents=True)
    (db / "ASVspoof2019_LA_cm_protocols" / "ASVspoof2019.LA.cm.train.trn.txt").write_text("\n".join(g["protocol"]) + "\n")
    flac = db / "ASVspoof2019_LA_train" / "flac"
    flac.mkdir(parents=True)
    for i, k in enumerate(g["keys"]):
        (flac / f"{k}.flac").write_bytes(encode(dirty_audio(i).astype(np.int64), plan=lambda f, c, b: {"kind": "verbatim"}))
    conf = tmp_path / "toy.conf"
    conf.write_text(json.dumps({"database_path": str(db), "track": "LA", "model_config": {"architecture": "ToyScore"}}))
    mp = tmp_path / "toy.pth"
    torch.save({"module.w": torch.tensor(g["weights"])}, mp)
    out = tmp_path / "dirty_samples.txt"
    fdd.main(fdd.parse_args(["--config", str(conf), "--model_path", str(mp), "--output_path", str(out),
                             "--batch_size", str(g["batch_size"]), "--filter_ratio", str(g["filter_ratio"]),
                             "--device", "cuda", "--seed", str(g["np_seed"])]))
    assert (tmp_path / "dirty_samples_cleaned_protocol.txt").read_text() == g["cleaned_protocol_txt"]
    got = [ln.split() for ln in out.read_text().splitlines()]
    ref = [ln.split() for ln in g["dirty_txt"].splitlines()]
    assert [(a[0], a[2]) for a in got] == [(b[0], b[2]) for b in ref]
    np.testing.assert_allclose([float(a[1]) for a in got], [float(b[1]) for b in ref], rtol=0, atol=3e-6)
