"""Deterministic, construction-order-independent parameter fill shared by the golden generator
(run against the reference modules) and the tests (run against the oracle / product modules).

Every floating tensor of a state_dict is filled from numpy's PCG64 seeded by (seed, crc32(key)),
so two modules with the same state_dict keys and shapes get identical values whatever order they
create their parameters in. Fixtures then only need to store inputs and outputs.
"""
import zlib

import numpy as np
import torch


def _value(key, shape, seed):
    rng = np.random.default_rng([seed, zlib.crc32(key.encode())])
    n = int(np.prod(shape)) if len(shape) else 1
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "running_var":
        v = rng.uniform(0.5, 1.5, n)
    elif leaf == "running_mean":
        v = rng.normal(0.0, 0.2, n)
    elif leaf == "A_log":
        d_state = shape[-1]
        v = (np.log(np.tile(np.arange(1, d_state + 1, dtype=np.float64), n // d_state))
             + rng.normal(0.0, 0.05, n))
    elif leaf == "D" or (leaf == "weight" and len(shape) == 1) or leaf in ("weight_g", "original0"):
        v = 1.0 + rng.normal(0.0, 0.1, n)
    elif leaf == "bias" or len(shape) <= 1:
        v = rng.normal(0.0, 0.1, n)
    else:
        fan_in = n // shape[0]
        v = rng.normal(0.0, 1.0 / np.sqrt(max(fan_in, 1)), n)
    return v.reshape(shape)


def seeded_fill_(module, seed=1234, skip=()):
    """Fill module's parameters and float buffers in place; returns the list of keys filled."""
    sd = module.state_dict()
    done = []
    with torch.no_grad():
        for k in sorted(sd.keys()):
            t = sd[k]
            if not torch.is_floating_point(t) or any(s in k for s in skip):
                continue
            t.copy_(torch.from_numpy(_value(k, tuple(t.shape), seed)).to(t.dtype))
            done.append(k)
    return done


def seeded_array(tag, shape, seed=1234, scale=1.0):
    rng = np.random.default_rng([seed, zlib.crc32(tag.encode())])
    return rng.standard_normal(shape) * scale


DIRTY_LENS = [30000, 70000, 64000, 100000, 30000, 50000, 66000, 20000, 30000, 90000, 64601, 45000] * 3


def dirty_audio(i):
    """Utterance i of the dirty-filter fixture as int16 samples (FLAC-encodable, and what sf.read returns
    divided by 32768). Utterances 0, 4 and 8 (+12k) are identical and shorter than 64 600 samples, so their
    losses tie exactly and pin the stable order of the sort."""
    n = DIRTY_LENS[i]
    tie = i % 12 in (0, 4, 8)
    rng = np.random.default_rng(0 if tie else 100 + i)
    off = 0 if tie else 400 * (i % 5 - 2)
    return np.clip(np.round(3000 * rng.standard_normal(n) + off), -32768, 32767).astype(np.int16)
