"""Dirty-data filter host logic (radhip/dirty.py) against the reference's own run
(tests/golden/dirty_filter.json, make_golden.gen_dirty: src/filter_dirty_data.py on a toy scorer): fed the
per-utterance losses the reference computed, the stable descending sort, the int(N * ratio) cut and the
two writers reproduce the reference's dirty list and cleaned protocol byte for byte (including the
tie order of identical utterances). The GPU scoring pass itself is tests/test_dirty_gpu.py."""
import numpy as np


def test_select_and_write_reproduce_reference_bytes(golden, tmp_path):
    from radhip.dirty import protocol_line_map, select_dirty, write_outputs
    g = golden("dirty_filter.json")
    proto = tmp_path / "trn.txt"
    proto.write_text("\n".join(g["protocol"]) + "\n")
    labels = [1 if ln.split()[-1] == "bonafide" else 0 for ln in g["protocol"]]
    losses = np.asarray(g["losses"], dtype=np.float32)
    dirty, clean = select_dirty(g["keys"], losses, labels, np.zeros(len(labels)), g["filter_ratio"])
    assert len(dirty) == int(len(labels) * g["filter_ratio"])
    out = tmp_path / "dirty_samples.txt"
    clean_path = write_outputs(out, dirty, clean, protocol_line_map(proto))
    assert clean_path == str(tmp_path / "dirty_samples_cleaned_protocol.txt")
    assert out.read_text() == g["dirty_txt"]
    assert (tmp_path / "dirty_samples_cleaned_protocol.txt").read_text() == g["cleaned_protocol_txt"]


def test_unknown_key_gets_the_reference_fallback_line(tmp_path):
    from radhip.dirty import write_outputs
    p = write_outputs(tmp_path / "x.txt", [], [{"file": "LA_T_1", "loss": 0.1, "label": 1, "prob": 0.9},
                                               {"file": "LA_T_2", "loss": 0.0, "label": 0, "prob": 0.9}], {})
    assert p == str(tmp_path / "x_cleaned_protocol.txt")
    assert open(p).read() == "LA_0000 LA_T_1 - - bonafide\nLA_0000 LA_T_2 - - spoof\n"


def test_ratio_below_one_sample_keeps_everything():
    from radhip.dirty import select_dirty
    dirty, clean = select_dirty(["a", "b"], [0.5, 0.7], [0, 1], [0.5, 0.5], 0.02)
    assert dirty == [] and [r["file"] for r in clean] == ["b", "a"]
