"""Per-utterance augmentation API (radhip.augment) on the GPU: the reference's RawBoost(algo_id, fs).process
(src/rawboost.py:9-33) and apply_codec_aug (src/data_utils.py:31-59), checked against the oracle
(oracle/rawboost.py, pinned to the reference by tests/golden/rawboost.npz; oracle/resample.py, the
torchaudio restatement) on the same seeds, including the host RNG each call consumes."""
import random

import numpy as np
import pytest
import torch

from seeded import seeded_array

pytestmark = pytest.mark.gpu


def test_rawboost_process_lnl_equals_oracle():
    from oracle import rawboost as orb
    from radhip.augment import RawBoost
    x = seeded_array("aug.lnl", (48000,), scale=0.1).astype(np.float32).astype(np.float64)
    np.random.seed(5)
    got = RawBoost(algo_id=[1]).process(x)
    after = np.random.get_state()[1].copy()
    np.random.seed(5)
    ref = orb.process(x, [1])
    assert got.dtype == np.float64 and got.shape == x.shape
    np.testing.assert_allclose(got, ref, rtol=2e-6, atol=2e-7 * np.abs(ref).max())
    np.testing.assert_array_equal(after, np.random.get_state()[1])     # same numpy draws consumed


@pytest.mark.parametrize("algo", [2, 3, 4])
def test_rawboost_process_noise_algorithms_equal_oracle(algo):
    """ISD / SSI: the per-utterance API draws the reference's own noise (randn + choice / randn before the SNR,
    src/rawboost.py:66-95) from numpy's global RNG, so output and RNG state equal the oracle's (pinned to the
    reference by tests/golden/rawboost.npz) on the same seed."""
    from oracle import rawboost as orb
    from radhip.augment import RawBoost
    x = seeded_array(f"aug.noise{algo}", (48011,), scale=0.1).astype(np.float32).astype(np.float64)
    np.random.seed(9 + algo)
    got = RawBoost(algo_id=[algo]).process(x)
    after = np.random.get_state()[1].copy()
    np.random.seed(9 + algo)
    ref = orb.process(x, [algo])
    np.testing.assert_array_equal(after, np.random.get_state()[1])     # same numpy draws consumed
    assert got.dtype == np.float64 and got.shape == x.shape
    # fp64 on the device, rounded to fp32 once at the end (the model's input dtype)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-7 * np.abs(ref).max())


@pytest.mark.parametrize("algo", [2, 3, 4])
def test_rawboost_process_philox_mode(algo):
    """exact=False: the batched train path's draw (one Philox seed per ISD / SSI call, documented deviation):
    same numpy draws as Augmenter's, the effect has the reference's statistics."""
    from radhip.augment import RawBoost, draw_rawboost
    n = 64000
    x = np.full(n, 0.1)
    np.random.seed(9)
    got = RawBoost(algo_id=[algo], exact=False).process(x)
    after = np.random.get_state()[1].copy()
    np.random.seed(9)
    np.random.randint(0, 1)
    rec = draw_rawboost(n, algo)
    np.testing.assert_array_equal(after, np.random.get_state()[1])
    if algo == 2:
        frac = np.mean(got != np.float32(0.1))
        assert abs(frac - 1.0 / rec.beta) < 0.01
    elif algo == 3:
        snr = 10 * np.log10(np.sum(x ** 2) / np.sum((got - 0.1) ** 2))
        assert abs(snr - rec.snr_db) < 0.01
    else:
        assert np.isfinite(got).all() and not np.allclose(got, x)


def test_augmenter_exact_noise_equals_oracle():
    """The batched train path with exact_noise: every utterance of a micro-batch (algo 5 = uniform over 1-4,
    ragged lengths incl. one shorter than 64 600, RawBoost p 1, codec off) equals the oracle's per-utterance
    RawBoost + pad_random on the same numpy / python seeds, and the RNG streams end in the same state."""
    import random as pyrandom
    from oracle import rawboost as orb
    from oracle.data import pad_random
    from radhip.train import Augmenter
    lens = [70001, 64601, 52000, 66000, 80000, 64700]
    xs = [seeded_array(f"aug.batch{i}", (n,), scale=0.1).astype(np.float32) for i, n in enumerate(lens)]
    aug = Augmenter("cuda", algo=5, rawboost_p=1.0, use_codec=False, exact_noise=True)
    flat = torch.from_numpy(np.concatenate(xs)).cuda()
    offs = list(np.cumsum([0] + lens[:-1]))
    np.random.seed(21)
    pyrandom.seed(21)
    plan = aug.draw(lens)
    got = aug.run(flat, offs, lens, plan).cpu().numpy()
    st_np, st_py = np.random.get_state()[1].copy(), pyrandom.getstate()
    np.random.seed(21)
    pyrandom.seed(21)
    refs = []
    for x in xs:                       # __getitem__ order: RawBoost gate (python), process (numpy), pad_random
        assert pyrandom.random() < 1.0
        y = orb.process(x.astype(np.float64), [1, 2, 3, 4])
        refs.append(pad_random(y))
    np.testing.assert_array_equal(st_np, np.random.get_state()[1])
    assert st_py == pyrandom.getstate()
    for b, ref in enumerate(refs):
        np.testing.assert_allclose(got[b], ref.astype(np.float32), rtol=1e-6, atol=1e-7 * np.abs(ref).max(),
                                   err_msg=f"utterance {b}")


def test_rawboost_process_none_returns_input():
    from radhip.augment import RawBoost
    x = np.ones(100)
    np.random.seed(1)
    assert RawBoost(algo_id=[0]).process(x) is x


@pytest.mark.parametrize("seed", [0, 1, 3, 8])
def test_apply_codec_aug_equals_oracle_roundtrip(seed):
    from oracle.resample import resample
    from radhip.augment import apply_codec_aug
    x = seeded_array(f"aug.codec{seed}", (23001,), scale=0.1).astype(np.float32)
    random.seed(seed)
    got = apply_codec_aug(x)
    state = random.getstate()
    random.seed(seed)
    taken = random.random() < 0.5
    sr = random.choice([8000, 6000, 4000]) if taken else None
    assert random.getstate() == state
    if not taken:
        assert got is x
        return
    ref = resample(resample(x.astype(np.float64), 16000, sr), sr, 16000)
    assert got.dtype == np.float32 and got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=0, atol=4e-6)
