"""EER / t-DCF / min-flip EER restatements.

The EER is computed with plain Python (stable sort + explicit FRR/FAR sweep), independently of the
product's vectorised numpy version, restating compute_det_curve / compute_eer
(src/evaluation.py:126-160); the t-DCF restates calculate_tDCF_EER / obtain_asv_error_rates /
compute_tDCF (src/evaluation.py:7-123,163-335); min-flip restates compute_eer_minflip
(src/report_2021df_codec_breakdown.py:10-37). Pinned by tests/golden (B01/B02 known answers).
"""
import numpy as np


def det_curve(target, nontarget):
    """Lists (frr, far, thresholds) exactly as compute_det_curve builds them."""
    target = [float(v) for v in target]
    nontarget = [float(v) for v in nontarget]
    allsc = [(s, 1) for s in target] + [(s, 0) for s in nontarget]
    order = sorted(range(len(allsc)), key=lambda i: allsc[i][0])     # stable == numpy mergesort
    nt, nn = len(target), len(nontarget)
    frr, far = [0.0], [1.0]
    thr = [allsc[order[0]][0] - 0.001]
    tar_sum = 0
    for k, i in enumerate(order, start=1):
        tar_sum += allsc[i][1]
        frr.append(tar_sum / nt)
        far.append((nn - (k - tar_sum)) / nn)
        thr.append(allsc[i][0])
    return frr, far, thr


def compute_eer(target, nontarget):
    frr, far, thr = det_curve(target, nontarget)
    best, bi = None, 0
    for i, (a, b) in enumerate(zip(frr, far)):
        d = abs(a - b)
        if best is None or d < best:
            best, bi = d, i
    return (frr[bi] + far[bi]) / 2.0, thr[bi]


def compute_eer_minflip(bona, spoof):
    """Percent; min over the score sign (report_2021df_codec_breakdown.py:10-37)."""
    bona = np.asarray(bona, dtype=np.float64)
    spoof = np.asarray(spoof, dtype=np.float64)
    if bona.size == 0 or spoof.size == 0:
        return float("nan")
    e1 = compute_eer(bona, spoof)[0]
    e2 = compute_eer(-bona, -spoof)[0]
    return 100.0 * min(e1, e2)


COST_MODEL = {"Pspoof": 0.05, "Ptar": 0.95 * 0.99, "Pnon": 0.95 * 0.01, "Cmiss": 1, "Cfa": 10,
              "Cmiss_asv": 1, "Cfa_asv": 10, "Cmiss_cm": 1, "Cfa_cm": 10}


def min_tdcf(bona_cm, spoof_cm, tar_asv, non_asv, spoof_asv, cost=COST_MODEL):
    """Legacy ASVspoof-2019 normalised min t-DCF with the ASV threshold at its EER point."""
    _, thr = compute_eer(tar_asv, non_asv)
    tar_asv, non_asv, spoof_asv = map(np.asarray, (tar_asv, non_asv, spoof_asv))
    pfa_asv = np.sum(non_asv >= thr) / non_asv.size
    pmiss_asv = np.sum(tar_asv < thr) / tar_asv.size
    pmiss_spoof_asv = np.sum(spoof_asv < thr) / spoof_asv.size
    frr, far, _ = det_curve(bona_cm, spoof_cm)
    frr, far = np.asarray(frr), np.asarray(far)
    c1 = cost["Ptar"] * (cost["Cmiss_cm"] - cost["Cmiss_asv"] * pmiss_asv) - cost["Pnon"] * cost["Cfa_asv"] * pfa_asv
    c2 = cost["Cfa_cm"] * cost["Pspoof"] * (1 - pmiss_spoof_asv)
    t = (c1 * frr + c2 * far) / min(c1, c2)
    return float(t[int(np.argmin(t))])
