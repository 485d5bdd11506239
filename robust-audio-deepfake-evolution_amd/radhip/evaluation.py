"""Scoring: EER, legacy ASVspoof-2019 min t-DCF, 2021-DF min-flip EER with codec/source breakdown.

Vectorised numpy with the reference's exact operation order, so results are bit-identical to
src/evaluation.py and src/report_2021df_codec_breakdown.py:
* det_curve / eer follow compute_det_curve / compute_eer (src/evaluation.py:126-160): stable
  mergesort of the concatenated scores, cumulative FRR/FAR, argmin |FRR - FAR| (first index on ties);
* tdcf_curve / calculate_tDCF_EER follow src/evaluation.py:7-123,163-335 (C1/C2 weights, ASV
  threshold at the ASV EER point, legacy normalisation by min(C1, C2)); the report text matches
  byte for byte;
* eer_minflip, load_scores, parse_key_line and report_2021df follow
  src/report_2021df_codec_breakdown.py:10-146.

`calculate_EER_2021` fills the reference's missing 2021-DF scoring hook (src/main.py:36,368): overall
min-flip EER plus the per-codec breakdown, written as text.
"""
from collections import defaultdict
from dataclasses import dataclass
from pathlib import Path

import numpy as np

ATTACKS_2019 = tuple(f"A{i:02d}" for i in range(7, 20))


@dataclass(frozen=True)
class CostModel:
    """Legacy ASVspoof-2019 t-DCF parameters (src/evaluation.py:19-31)."""
    Pspoof: float = 0.05
    Cmiss_asv: float = 1.0
    Cfa_asv: float = 10.0
    Cmiss_cm: float = 1.0
    Cfa_cm: float = 10.0

    @property
    def Ptar(self):
        return (1 - self.Pspoof) * 0.99

    @property
    def Pnon(self):
        return (1 - self.Pspoof) * 0.01


def det_curve(target, nontarget):
    """(frr, far, thresholds), each of length n+1; threshold 0 is the lowest score - 0.001."""
    target = np.asarray(target)
    nontarget = np.asarray(nontarget)
    scores = np.concatenate((target, nontarget))
    is_target = np.concatenate((np.ones(target.size), np.zeros(nontarget.size)))
    order = np.argsort(scores, kind="mergesort")
    tar_cum = np.cumsum(is_target[order])
    non_cum = nontarget.size - (np.arange(1, scores.size + 1) - tar_cum)
    frr = np.concatenate((np.atleast_1d(0), tar_cum / target.size))
    far = np.concatenate((np.atleast_1d(1), non_cum / nontarget.size))
    thr = np.concatenate((np.atleast_1d(scores[order[0]] - 0.001), scores[order]))
    return frr, far, thr


def eer(target, nontarget):
    """(EER as a fraction, threshold at the EER point)."""
    frr, far, thr = det_curve(target, nontarget)
    k = np.argmin(np.abs(frr - far))
    return np.mean((frr[k], far[k])), thr[k]


def asv_error_rates(tar_asv, non_asv, spoof_asv, threshold):
    """(Pfa_asv, Pmiss_asv, Pmiss_spoof_asv) at a fixed ASV threshold (src/evaluation.py:111-123)."""
    pfa = sum(non_asv >= threshold) / non_asv.size
    pmiss = sum(tar_asv < threshold) / tar_asv.size
    pmiss_spoof = None if spoof_asv.size == 0 else np.sum(spoof_asv < threshold) / spoof_asv.size
    return pfa, pmiss, pmiss_spoof


class TDCFError(ValueError):
    pass


def tdcf_curve(bona_cm, spoof_cm, pfa_asv, pmiss_asv, pmiss_spoof_asv, cost=CostModel()):
    """Normalised t-DCF over every CM threshold, and the thresholds. Raises TDCFError where the
    reference calls sys.exit (missing spoof miss rate, nan/inf scores, < 3 distinct scores,
    negative weights)."""
    if pmiss_spoof_asv is None:
        raise TDCFError("the ASV miss rate on spoof trials is required")
    both = np.concatenate((bona_cm, spoof_cm))
    if np.isnan(both).any() or np.isinf(both).any():
        raise TDCFError("scores contain nan or inf")
    if np.unique(both).size < 3:
        raise TDCFError("soft CM scores are required, not binary decisions")
    pmiss_cm, pfa_cm, thr = det_curve(bona_cm, spoof_cm)
    c1 = cost.Ptar * (cost.Cmiss_cm - cost.Cmiss_asv * pmiss_asv) - cost.Pnon * cost.Cfa_asv * pfa_asv
    c2 = cost.Cfa_cm * cost.Pspoof * (1 - pmiss_spoof_asv)
    if c1 < 0 or c2 < 0:
        raise TDCFError("negative t-DCF weights: check the ASV error rates")
    return (c1 * pmiss_cm + c2 * pfa_cm) / np.minimum(c1, c2), thr


def _read_columns(path):
    return np.genfromtxt(path, dtype=str)


def tdcf_report(eer_cm, min_tdcf, eer_per_attack):
    """The text block calculate_tDCF_EER writes (src/evaluation.py:92-105)."""
    out = ["\nCM SYSTEM\n", "\tEER\t\t= {:8.9f} % (Equal error rate for countermeasure)\n".format(eer_cm * 100),
           "\nTANDEM\n", "\tmin-tDCF\t\t= {:8.9f}\n".format(min_tdcf), "\nBREAKDOWN CM SYSTEM\n"]
    for a, e in eer_per_attack.items():
        out.append(f"\tEER {a}\t\t= {e * 100:8.9f} % (Equal error rate for {a}\n")
    return "".join(out)


def calculate_tDCF_EER(cm_scores_file, asv_score_file, output_file, printout=True, cost=CostModel()):
    """CM score file ("utt src key score") + organiser ASV scores ("spk key score") ->
    (EER %, min t-DCF); writes the report when printout (src/evaluation.py:7-108)."""
    asv = _read_columns(asv_score_file)
    asv_keys, asv_scores = asv[:, 1], asv[:, 2].astype(np.float64)
    cm = _read_columns(cm_scores_file)
    cm_src, cm_keys, cm_scores = cm[:, 1], cm[:, 2], cm[:, 3].astype(np.float64)
    tar_asv = asv_scores[asv_keys == "target"]
    non_asv = asv_scores[asv_keys == "nontarget"]
    spoof_asv = asv_scores[asv_keys == "spoof"]
    bona_cm = cm_scores[cm_keys == "bonafide"]
    spoof_cm = cm_scores[cm_keys == "spoof"]
    _, asv_thr = eer(tar_asv, non_asv)
    eer_cm = eer(bona_cm, spoof_cm)[0]
    curve, _ = tdcf_curve(bona_cm, spoof_cm, *asv_error_rates(tar_asv, non_asv, spoof_asv, asv_thr), cost)
    min_tdcf = curve[np.argmin(curve)]
    if printout:
        per_attack = {a: eer(bona_cm, cm_scores[cm_src == a])[0] for a in ATTACKS_2019}
        text = tdcf_report(eer_cm, min_tdcf, per_attack)
        Path(output_file).write_text(text)
        print(text, end="")
    return eer_cm * 100, min_tdcf


def eer_minflip(bona, spoof):
    """EER in % as min over the score sign (src/report_2021df_codec_breakdown.py:10-37); nan if a side
    is empty."""
    bona = np.asarray(bona, dtype=np.float64)
    spoof = np.asarray(spoof, dtype=np.float64)
    if bona.size == 0 or spoof.size == 0:
        return float("nan")
    labels = np.concatenate([np.ones_like(bona), np.zeros_like(spoof)]).astype(np.int64)
    scores = np.concatenate([bona, spoof])

    def one(sc):
        lab = labels[np.argsort(sc, kind="mergesort")]
        tar = lab.sum()
        non = lab.size - tar
        tar_cum = np.cumsum(lab)
        non_cum = non - (np.arange(1, lab.size + 1) - tar_cum)
        frr = np.concatenate(([0.0], tar_cum / max(tar, 1)))
        far = np.concatenate(([1.0], non_cum / max(non, 1)))
        k = np.argmin(np.abs(frr - far))
        return float(100.0 * 0.5 * (frr[k] + far[k]))

    return min(one(scores), one(-scores))


def load_scores(score_file):
    """{utt: score} from lines 'utt ... score'; unparsable lines skipped."""
    scores = {}
    with open(score_file) as f:
        for line in f:
            parts = line.split()
            if len(parts) < 2:
                continue
            try:
                scores[parts[0]] = float(parts[-1])
            except ValueError:
                continue
    return scores


@dataclass
class KeyRow:
    codec: str
    source: str
    key: str


def parse_key_line(parts):
    """trial_metadata.txt: SPK FILE CODEC SRC ATTACK KEY ... -> (FILE, KeyRow)."""
    return parts[1], KeyRow(codec=parts[2], source=parts[3], key=parts[5])


def group_scores_2021(scores, key_file):
    """Overall / per-codec / per-source bona-fide and spoof score lists for the scored trials."""
    groups = {"all": (defaultdict(list), defaultdict(list)), "codec": (defaultdict(list), defaultdict(list)),
              "source": (defaultdict(list), defaultdict(list))}
    with open(key_file) as f:
        for line in f:
            parts = line.split()
            if len(parts) < 6:
                continue
            utt, row = parse_key_line(parts)
            if utt not in scores:
                continue
            side = 0 if row.key == "bonafide" else 1
            s = scores[utt]
            groups["all"][side][""].append(s)
            groups["codec"][side][row.codec].append(s)
            groups["source"][side][row.source].append(s)
    return groups


def _breakdown_rows(bona, spoof):
    rows = []
    for name in sorted(set(bona) | set(spoof)):
        b = np.array(bona.get(name, []), dtype=np.float64)
        s = np.array(spoof.get(name, []), dtype=np.float64)
        e = eer_minflip(b, s) if (b.size > 0 and s.size > 0) else float("nan")
        rows.append((name, e, b.size, s.size))
    return rows


def report_2021df(score_file, key_file, out=None):
    """Markdown report of report_2021df_codec_breakdown.main; returns (text, overall EER %)."""
    g = group_scores_2021(load_scores(score_file), key_file)
    bona = np.array(g["all"][0][""], dtype=np.float64)
    spoof = np.array(g["all"][1][""], dtype=np.float64)
    overall = eer_minflip(bona, spoof)
    lines = ["# ASVspoof 2021 DF Report (Codec Breakdown)\n", f"- **Score file**: `{Path(score_file)}`",
             f"- **Key file**: `{Path(key_file)}`", f"- **Total bonafide**: {bona.size}",
             f"- **Total spoof**: {spoof.size}", f"- **Overall EER (minflip)**: **{overall:.3f}%**\n"]
    for title, head, key in (("## Breakdown by Codec\n", "| Codec |", "codec"),
                             ("\n## Breakdown by Source Domain\n", "| Source |", "source")):
        lines += [title, f"{head} EER (%) | Bonafide | Spoof | Total |", "| :--- | ---: | ---: | ---: | ---: |"]
        for name, e, nb, ns in _breakdown_rows(*g[key]):
            lines.append(f"| {name} | {e:.3f} | {nb} | {ns} | {nb + ns} |")
    text = "\n".join(lines) + "\n"
    if out is not None:
        Path(out).write_text(text, encoding="utf-8")
    return text, overall


def calculate_EER_2021(cm_scores_file, key_file, output_file, printout=True):
    """2021-DF scoring hook the reference calls but does not define (src/main.py:36,368,746).
    Returns (overall min-flip EER %, {codec: EER %})."""
    g = group_scores_2021(load_scores(cm_scores_file), key_file)
    overall = eer_minflip(g["all"][0][""], g["all"][1][""])
    per_codec = {name: e for name, e, _, _ in _breakdown_rows(*g["codec"])}
    text = "\nCM SYSTEM (ASVspoof 2021 DF)\n\tEER\t\t= {:8.9f} % (min over score sign)\n".format(overall)
    text += "\nBREAKDOWN BY CODEC\n" + "".join(f"\tEER {k}\t\t= {v:8.9f} %\n" for k, v in per_codec.items())
    Path(output_file).write_text(text)
    if printout:
        print(text, end="")
    return overall, per_codec
