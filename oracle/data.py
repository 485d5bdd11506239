"""Protocol parsing and padding restatements (plain Python / numpy).

Restates genSpoof_list (src/data_utils.py:62-104), pad (:107-113) and pad_random (:116-127).
"""
import numpy as np


def gen_spoof_list(lines, is_train=False, is_eval=False, is_2021=False):
    """Same return structure as genSpoof_list: 2021 -> list; train/dev -> (labels, list); eval -> list."""
    if is_2021:
        out = []
        for ln in lines:
            ln = ln.strip()
            if not ln:
                continue
            parts = ln.split()
            out.append(parts[1] if len(parts) >= 2 else parts[0])
        return out
    keys, labels = [], {}
    for ln in lines:
        _, key, _, _, lab = ln.strip().split(" ")
        keys.append(key)
        if not is_eval:
            labels[key] = 1 if lab == "bonafide" else 0
    if is_eval and not is_train:
        return keys
    return labels, keys


def pad(x, max_len=64600):
    x = np.asarray(x)
    n = x.shape[0]
    if n >= max_len:
        return x[:max_len]
    reps = int(max_len / n) + 1
    return np.tile(x, (1, reps))[:, :max_len][0]


def pad_random(x, max_len=64600, rng=np.random):
    """Crops at rng.randint(len - max_len) (raises for len == max_len, as the reference does)."""
    x = np.asarray(x)
    n = x.shape[0]
    if n >= max_len:
        s = rng.randint(n - max_len)
        return x[s:s + max_len]
    reps = int(max_len / n) + 1
    return np.tile(x, reps)[:max_len]
