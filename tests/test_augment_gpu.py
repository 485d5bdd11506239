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
def test_rawboost_process_noise_algorithms(algo):
    """ISD / SSI noise comes from the device Philox stream (documented deviation): the numpy draws
    consumed are those of the batched path (Augmenter), the effect has the reference's statistics."""
    from radhip.augment import RawBoost, draw_rawboost
    n = 64000
    x = np.full(n, 0.1)
    np.random.seed(9)
    got = RawBoost(algo_id=[algo]).process(x)
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
