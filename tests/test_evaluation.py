"""Product scoring (radhip.evaluation / radhip.infer) against the reference's golden outputs (CPU)."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from radhip import evaluation as EV
from radhip.infer import produce_evaluation_file, produce_evaluation_file_sharded, shard_bounds

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["B01", "B02"])
def test_eer_subsample_bit_exact(name):
    s = _json("eval_golden.json")[name]["subsample"]
    e, t = EV.eer(np.array(s["bona"]), np.array(s["spoof"]))
    assert float(e) == s["eer"] and float(t) == s["thr"]
    assert EV.eer_minflip(s["bona"], s["spoof"]) == s["minflip_pct"]


def test_eer_matches_oracle_with_ties():
    from oracle.evaluation import compute_eer
    rng = np.random.default_rng(0)
    for _ in range(5):
        b = np.round(rng.normal(1, 1, 300), 1)
        s = np.round(rng.normal(-1, 1, 900), 1)
        e, t = EV.eer(b, s)
        eo, to = compute_eer(b, s)
        assert float(e) == pytest.approx(eo, abs=0) and float(t) == to


def test_tdcf_report_bytes(tmp_path):
    g = _json("eval_golden.json")["tdcf"]
    cm, asv, rep = tmp_path / "cm.txt", tmp_path / "asv.txt", tmp_path / "rep.txt"
    cm.write_text("\n".join(g["cm_lines"]) + "\n")
    asv.write_text("\n".join(g["asv_lines"]) + "\n")
    eer_pct, tdcf = EV.calculate_tDCF_EER(cm, asv, rep, printout=True)
    assert eer_pct == g["eer_cm_pct"] and tdcf == g["min_tdcf"]
    assert rep.read_text() == g["report"]
    # printout=False returns the same numbers and writes nothing
    rep.unlink()
    assert EV.calculate_tDCF_EER(cm, asv, rep, printout=False) == (eer_pct, tdcf)
    assert not rep.exists()


def test_tdcf_rejects_binary_scores():
    with pytest.raises(EV.TDCFError):
        EV.tdcf_curve(np.array([1.0, 1.0]), np.array([0.0, 0.0]), 0.01, 0.02, 0.5)
    with pytest.raises(EV.TDCFError):
        EV.tdcf_curve(np.array([1.0, np.nan, 2.0]), np.array([0.0, 3.0]), 0.01, 0.02, 0.5)


def test_report_2021df_bytes(tmp_path, monkeypatch):
    g = _json("eval21_golden.json")
    monkeypatch.chdir(tmp_path)
    open("trial_metadata.txt", "w").write("\n".join(g["meta"]) + "\n")
    open("scores.txt", "w").write("\n".join(g["scores"]) + "\n")
    text, overall = EV.report_2021df("scores.txt", "trial_metadata.txt", out="report.md")
    assert text == g["report"]
    assert open("report.md").read() == g["report"]
    eer, per_codec = EV.calculate_EER_2021("scores.txt", "trial_metadata.txt", "eer.txt", printout=False)
    assert eer == overall and "low_mp3" in per_codec and os.path.exists("eer.txt")


def test_minflip_empty_side_is_nan():
    assert np.isnan(EV.eer_minflip([], [1.0, 2.0]))


class _Toy(torch.nn.Module):
    def __init__(self, w):
        super().__init__()
        self.w = torch.nn.Parameter(torch.from_numpy(w))

    def forward(self, xb, Freq_aug=False):
        return xb, xb @ self.w


def test_score_file_bytes(tmp_path):
    g = np.load(os.path.join(GOLD, "scorefile.npz"), allow_pickle=False)
    x, trial = g["x"], str(g["trial"]).split("\n")
    ids = [t.split()[1] for t in trial]
    tp, sp = tmp_path / "trl.txt", tmp_path / "score.txt"
    tp.write_text("\n".join(trial) + "\n")
    batches = [(torch.from_numpy(x[i:i + 8]), ids[i:i + 8]) for i in range(0, len(ids), 8)]
    produce_evaluation_file(batches, _Toy(g["w"]), torch.device("cpu"), sp, tp)
    assert sp.read_text() == str(g["text"])


def test_score_file_order_mismatch_raises(tmp_path):
    g = np.load(os.path.join(GOLD, "scorefile.npz"), allow_pickle=False)
    trial = str(g["trial"]).split("\n")
    tp = tmp_path / "trl.txt"
    tp.write_text("\n".join(trial) + "\n")
    ids = [t.split()[1] for t in trial][::-1]
    batches = [(torch.from_numpy(g["x"]), ids)]
    with pytest.raises(AssertionError):
        produce_evaluation_file(batches, _Toy(g["w"]), torch.device("cpu"), tmp_path / "s.txt", tp)


def test_shard_bounds_cover():
    for n in (0, 1, 7, 37, 71237):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


class _DS:
    def __init__(self, x, ids):
        self.x, self.ids = x, ids

    def __len__(self):
        return len(self.ids)

    def __getitem__(self, i):
        return torch.from_numpy(self.x[i]), self.ids[i]


def _shard_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = np.load(os.path.join(GOLD, "scorefile.npz"), allow_pickle=False)
        trial = str(g["trial"]).split("\n")
        tp = os.path.join(out, "trl.txt")
        if rank == 0:
            open(tp, "w").write("\n".join(trial) + "\n")
        dist.barrier()
        ds = _DS(g["x"], [t.split()[1] for t in trial])
        produce_evaluation_file_sharded(ds, _Toy(g["w"]), torch.device("cpu"), os.path.join(out, "score.txt"), tp,
                                        batch_size=5)
    finally:
        dist.destroy_process_group()


def test_sharded_score_file_equals_single_process():
    """3 gloo ranks, contiguous shards, all_gather: the file is byte-identical to the reference's."""
    g = np.load(os.path.join(GOLD, "scorefile.npz"), allow_pickle=False)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_shard_worker, args=(3, port, out), nprocs=3, join=True, start_method="spawn")
        assert open(os.path.join(out, "score.txt")).read() == str(g["text"])
