"""Data path on the CPU: native FLAC reader (libradio.so), protocol parsing, padding, CLI surface.

The FLAC reader is pinned by round trips through tests/flac_writer.py, an independent spec-driven
encoder (soundfile/libsndfile, the flac tool and any .flac fixture are absent from the image and from
the reference), covering every subframe and stereo mode; corruption must raise, as libsndfile does.
Protocol parsing is pinned to the reference-generated golden (tests/golden/protocol.json).
"""
import os

import numpy as np
import pytest

from flac_writer import encode


@pytest.fixture(scope="module")
def audio():
    from radhip import audio
    return audio


def _signal(n, seed=0, amp=3000, bits=16):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    x = amp * np.sin(t * 0.031) + 0.4 * amp * np.sin(t * 0.17) + rng.normal(0, amp / 20, n)
    lim = 2 ** (bits - 1)
    return np.clip(np.round(x), -lim, lim - 1).astype(np.int64)


def test_radio_exports_header_symbols(audio):
    L = audio.lib()
    syms = audio.header_symbols()
    assert len(syms) == 5
    for s in syms:
        assert hasattr(L, s), s


@pytest.mark.parametrize("kind", ["verbatim", "fixed0", "fixed1", "fixed2", "fixed3", "fixed4", "lpc"])
@pytest.mark.parametrize("method", [0, 1])
def test_flac_subframe_round_trip(audio, kind, method):
    x = _signal(9000, seed=len(kind) * 10 + method)
    data = encode(x, blocksize=4096, plan=lambda f, c, b: {"kind": kind, "porder": f % 4, "method": method})
    y, sr = audio.decode_bytes(data)
    assert sr == 16000 and y.dtype == np.float64 and y.shape == x.shape
    np.testing.assert_array_equal(y * 32768.0, x.astype(np.float64))


def test_flac_constant_wasted_escape_and_block_sizes(audio):
    x = _signal(5000, seed=5)
    x[:1152] = 77                                    # constant frame
    x[2304:3456] = (x[2304:3456] // 8) * 8           # 3 wasted bits
    plans = {0: {"kind": "constant"}, 1: {"kind": "lpc", "lpc_order": 32, "prec": 15, "porder": 3},
             2: {"kind": "fixed2", "wasted": 3, "porder": 2}, 3: {"kind": "fixed1", "escape_bits": 17},
             4: {"kind": "lpc", "lpc_order": 1, "method": 1}}
    data = encode(x, blocksize=1152, plan=lambda f, c, b: plans[f])
    y, _ = audio.decode_bytes(data)
    np.testing.assert_array_equal(y * 32768.0, x.astype(np.float64))
    for bs in (192, 200, 4096):                      # 8-bit/16-bit explicit and table block sizes
        y, _ = audio.decode_bytes(encode(x[:4500], blocksize=bs))
        np.testing.assert_array_equal(y * 32768.0, x[:4500].astype(np.float64))


@pytest.mark.parametrize("mode", ["independent", "left_side", "right_side", "mid_side"])
def test_flac_stereo_modes(audio, mode):
    L = _signal(6000, seed=1)
    R = _signal(6000, seed=2, amp=9000)
    x = np.stack([L, R], 1)
    y, _ = audio.decode_bytes(encode(x, stereo_mode=mode, plan=lambda f, c, b: {"kind": "lpc", "porder": 1}))
    assert y.shape == (6000, 2)
    np.testing.assert_array_equal(y * 32768.0, x.astype(np.float64))


def test_flac_24bit_normalisation(audio):
    x = _signal(3000, seed=4, amp=2 ** 21, bits=24)
    y, _ = audio.decode_bytes(encode(x, bps=24, plan=lambda f, c, b: {"kind": "fixed2", "method": 1}))
    np.testing.assert_array_equal(y * float(2 ** 23), x.astype(np.float64))


def test_flac_corruption_and_truncation_raise(audio):
    x = _signal(8192, seed=6)
    data = bytearray(encode(x))
    bad = bytearray(data)
    bad[len(bad) // 2] ^= 0x10                       # body bit flip -> CRC-16 mismatch
    with pytest.raises(audio.AudioReadError, match="corrupt"):
        audio.decode_bytes(bytes(bad))
    with pytest.raises(audio.AudioReadError):        # truncated stream: sample count != STREAMINFO
        audio.decode_bytes(bytes(data[:len(data) - 100]))
    with pytest.raises(audio.AudioReadError, match="not a FLAC"):
        audio.decode_bytes(b"RIFF" + bytes(100))


def test_flac_files_probe_read_and_batch(audio, tmp_path):
    paths, sigs = [], []
    for i, n in enumerate([64600, 70000, 12345, 64000]):
        x = _signal(n, seed=10 + i)
        p = tmp_path / f"u{i}.flac"
        data = encode(x, plan=lambda f, c, b: {"kind": ["lpc", "fixed2", "verbatim"][f % 3], "porder": f % 3})
        if i == 1:
            data = b"ID3\x03\x00\x00\x00\x00\x00\x0a" + bytes(10) + data   # ID3v2 tag in front
        p.write_bytes(data)
        paths.append(p)
        sigs.append(x)
    for p, x in zip(paths, sigs):
        fr, ch, sr, bits = audio.probe(p)
        assert (fr, ch, sr, bits) == (len(x), 1, 16000, 16)
        y, sr = audio.read(p)
        np.testing.assert_array_equal(y * 32768.0, x.astype(np.float64))
    buf, offs, lens = audio.read_batch(paths, threads=3)
    assert buf.dtype == np.float32 and list(lens) == [len(x) for x in sigs]
    for o, x in zip(offs, sigs):
        np.testing.assert_array_equal(buf[o:o + len(x)].astype(np.float64) * 32768.0, x.astype(np.float64))
    with pytest.raises(audio.AudioReadError):
        audio.read_batch(paths + [tmp_path / "missing.flac"])


def test_wav_read_matches_soundfile_normalisation(audio, tmp_path):
    from scipy.io import wavfile
    x = _signal(4000, seed=3).astype(np.int16)
    p = tmp_path / "a.wav"
    wavfile.write(p, 16000, x)
    y, sr = audio.read(p)
    assert sr == 16000
    np.testing.assert_array_equal(y, x.astype(np.float64) / 32768.0)


def test_genspoof_list_matches_reference_golden(golden, tmp_path):
    from radhip.data import genSpoof_list
    g = golden("protocol.json")
    tr = tmp_path / "train.txt"
    tr.write_text("\n".join(g["lines_train"]) + "\n")
    labels, keys = genSpoof_list(tr, is_train=True)
    assert keys == g["train"]["list"] and labels == g["train"]["labels"]
    labels, keys = genSpoof_list(tr, is_train=False, is_eval=False)
    assert keys == g["dev"]["list"] and labels == g["dev"]["labels"]
    assert genSpoof_list(tr, is_eval=True) == g["eval"]
    df = tmp_path / "df.txt"
    df.write_text("\n".join(g["lines_2021"]) + "\n")
    assert genSpoof_list(df, is_2021=True) == g["df2021"]


def test_pad_and_pad_random_match_oracle(golden):
    from oracle import data as od
    from radhip.data import pad, pad_random
    rng = np.random.default_rng(0)
    for n in (1000, 64599, 64601, 100000):
        x = rng.standard_normal(n)
        np.testing.assert_array_equal(pad(x), od.pad(x))
        np.random.seed(n)
        a = pad_random(x)
        np.random.seed(n)
        b = od.pad_random(x)
        np.testing.assert_array_equal(a, b)
    with pytest.raises(ValueError):          # the reference's randint(0) at len == 64600
        pad_random(rng.standard_normal(64600))


def test_cli_flags_and_output_layout(tmp_path):
    import main as cli
    a = cli.parse_args(["--config", "config/Phase6_Proposed.conf", "--comment", "x", "--eval",
                        "--eval_model_weights", "w.pth", "--seed", "7", "--start_epoch", "2"])
    assert a.eval and a.seed == 7 and a.start_epoch == 2 and a.eval_model_weights == "w.pth"
    assert a.output_dir == "./exp_result" and a.amp == "fp16" and not a.eager   # the reference's autocast dtype
    cfg = {"track": "LA", "num_epochs": 20, "batch_size": 8}
    assert str(cli.model_tag_dir(a, cfg)) == os.path.join("exp_result", "LA_Phase6_Proposed_ep20_bs8_x")
    from pathlib import Path
    trn, dev, ev = cli.protocol_paths({"data_config": {}}, "LA", Path("/db"))
    assert str(trn) == "/db/ASVspoof2019_LA_cm_protocols/ASVspoof2019.LA.cm.train.trn.txt"
    assert str(dev) == "/db/ASVspoof2019_LA_cm_protocols/ASVspoof2019.LA.cm.dev.trl.txt"
    assert str(ev) == "/db/ASVspoof2019_LA_cm_protocols/ASVspoof2019.LA.cm.eval.trl.txt"
    trn, _, _ = cli.protocol_paths({"data_config": {"custom_train_protocol": "/c/p.txt"}}, "LA", Path("/db"))
    assert str(trn) == "/c/p.txt"


def test_swa_running_mean():
    import torch
    import main as cli
    p = torch.nn.Parameter(torch.zeros(3))
    s = cli.SWA([p])
    for v in (1.0, 2.0, 6.0):
        p.data.fill_(v)
        s.update()
    s.swap()
    assert torch.allclose(p.data, torch.full((3,), 3.0))
    s.swap()
    assert torch.allclose(p.data, torch.full((3,), 6.0))


@pytest.mark.parametrize("n,B,world", [(20, 4, 1), (22, 4, 1), (37, 3, 2)])
def test_train_feeder_order_equals_reference_dataloader(n, B, world):
    """TrainFeeder's per-epoch order == the reference's DataLoader(shuffle=True, drop_last=True,
    generator=Generator().manual_seed(seed)) (src/main.py:909-920) over several epochs; with world > 1
    each rank takes its B-row share of every global batch of world * B."""
    import torch
    from torch.utils.data import DataLoader
    from radhip.data import TrainFeeder
    keys = [f"LA_T_{i:07d}" for i in range(n)]
    g = torch.Generator()
    g.manual_seed(1234)
    dl = DataLoader(keys, batch_size=B * world, shuffle=True, drop_last=True, generator=g)
    feeders = [TrainFeeder(keys, {k: 0 for k in keys}, "/nonexistent", B, None, 1234, rank=r, world=world)
               for r in range(world)]
    for _ in range(3):
        ref = [list(b) for b in dl]
        got = [list(f.epoch()) for f in feeders]
        for r in range(world):
            assert got[r] == [b[r * B:(r + 1) * B] for b in ref]


def test_getitem_gate_order_matches_reference(golden):
    """Dataset_ASVspoof2019_train.__getitem__ (data_utils.py:163-184) draw order, pinned by
    getitem_order.json (make_golden.gen_getitem runs the reference's own dataset, RawBoost algo 1):
    RawBoost gate and draws, codec gates and rate, then pad_random's crop start on the post-codec
    length — replayed call by call through Augmenter.draw on the same python / numpy seeds."""
    import random
    from radhip.train import Augmenter
    g = golden("getitem_order.json")
    aug = Augmenter("cpu", algo=g["algo"], rawboost_p=g["rawboost_p"], use_codec=g["use_codec"], codec_p=g["codec_p"])
    random.seed(g["seed"])
    np.random.seed(g["seed"])
    got = []
    for n, *_ in g["records"]:
        (rec, sr, start), = aug.draw([n])
        m = aug.codec_len(n, sr) if sr is not None else n
        got.append([n, int(rec is not None), sr or 0, start if m > aug.max_len else -1, m])
    assert got == g["records"]
    assert 0 < sum(r[1] for r in got) < len(got) and 0 < sum(1 for r in got if r[2]) < len(got)
