"""RawBoost restatement with the reference's exact numpy RNG consumption order.

Restates src/rawboost.py:3-95 (RawBoost.process, lnl_convolutive_noise, isd_additive_noise,
stationary_noise). The draw_* functions consume np.random in the same order as the reference
(so a seeded oracle run equals a seeded reference run bit for bit, checked by
tests/golden/rawboost.npz); the *_apply functions are pure, so the same draws can be handed to
the GPU kernels (rdx_rawboost_batch) for exact parity.
"""
import numpy as np
from scipy import signal


def _pick(seq, rng):
    return seq[rng.randint(0, len(seq))]            # rawboost.py:6-7 rand_list


def draw_lnl(rng=np.random, N_f=5, n_list=(1, 2, 3, 4, 5), a_min=10, a_max=100):
    """rawboost.py:36-50,55: n, (unused a), five 2-tap FIR factors, n IIR factors, then f."""
    n = _pick(list(n_list), rng)
    _pick(range(a_min, a_max), rng)                  # drawn and unused by the reference (:40)
    b = np.array([1.0])
    for _ in range(N_f):
        b = np.convolve(b, np.array([1.0, rng.uniform(-1, 1)]))
    a = np.array([1.0])
    for _ in range(n):
        a = np.convolve(a, np.array([1.0, rng.uniform(-0.1, 0.1)]))
    f = rng.randn()
    return {"n": n, "b": b, "a": a, "f": f}


def lnl_apply(x, p):
    """rawboost.py:52-63."""
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    lin = signal.lfilter(p["b"], p["a"], x)
    nl = lin + p["f"] * np.square(lin)
    rx = np.sqrt(np.mean(x ** 2))
    ra = np.sqrt(np.mean(nl ** 2))
    if ra == 0:
        return x
    return nl * (rx / ra)


def draw_isd(n, rng=np.random, P=10):
    """rawboost.py:67-73: beta, Gaussian noise, Bernoulli(1/beta) mask -> product noise*mask."""
    beta = _pick(range(5, P), rng)
    noise = rng.randn(n)
    mask = rng.choice([0, 1], size=n, p=[1 - 1 / beta, 1 / beta])
    return {"beta": beta, "nm": noise * mask}


def isd_apply(x, p, g_sd=2):
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    return x + g_sd * p["nm"] * x                    # rawboost.py:75


def draw_ssi(n, rng=np.random, snr_min=10, snr_max=40):
    """rawboost.py:82-88: Gaussian noise first, then the SNR."""
    noise = rng.randn(n)
    snr = rng.uniform(snr_min, snr_max)
    return {"noise": noise, "snr": snr}


def ssi_apply(x, p):
    """rawboost.py:84-95."""
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    sp = np.sum(x ** 2)
    npow = np.sum(p["noise"] ** 2)
    req = sp / (10 ** (p["snr"] / 10))
    return x + p["noise"] * np.sqrt(req / (npow + 1e-9))


def draw_process(n, algo_ids, rng=np.random):
    """RawBoost.process (rawboost.py:15-33): algorithm choice, then that algorithm's draws."""
    algo = _pick(list(algo_ids), rng)
    d = {"algo": algo}
    if algo in (1, 4):
        d["lnl"] = draw_lnl(rng)
    if algo in (2, 4):
        d["isd"] = draw_isd(n, rng)
    if algo == 3:
        d["ssi"] = draw_ssi(n, rng)
    return d


def apply_process(x, d):
    algo = d["algo"]
    if algo == 1:
        return lnl_apply(x, d["lnl"])
    if algo == 2:
        return isd_apply(x, d["isd"])
    if algo == 3:
        return ssi_apply(x, d["ssi"])
    if algo == 4:
        return isd_apply(lnl_apply(x, d["lnl"]), d["isd"])
    return np.asarray(x)


def process(x, algo_ids, rng=np.random):
    """Seeded drop-in of RawBoost(algo_ids).process(x)."""
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    return apply_process(x, draw_process(len(x), algo_ids, rng))
