"""The ensemble oracle (oracle/ensemble_oracle.py) against the reference's own
``derive_modalities`` / ``run_ensemble_inference`` outputs (tests/golden/
ensemble_fixtures.npz, made by gen_ensemble_fixtures.py), plus the product package's
bone tables (checked without a GPU)."""
import numpy as np
import pytest
import torch

import formula
from oracle import ensemble_oracle as eo
from oracle import model_oracle as mo

STREAMS = eo.MODALITIES


def oracle_models():
    models = {}
    for k, s in enumerate(STREAMS):
        m = mo.Model(num_class=2, num_point=33, num_person=1, graph="unused")
        formula.fill_state(m, seed=701 + 13 * k)
        models[s] = m.eval()
    return models


def test_bone_tables_match_reference(golden):
    from shiftgcn import ensemble as ens
    fx = golden("ensemble_fixtures.npz")
    assert [tuple(p) for p in fx["bone_pairs"]] == list(ens.MEDIAPIPE_BONE_PAIRS)
    assert tuple(fx["weights"]) == ens.ENSEMBLE_WEIGHTS_DEFAULT
    par = ens.parent_table(ens.MEDIAPIPE_BONE_PAIRS, 33)
    assert par[0] == 0 and par.dtype == np.int32
    ntu = ens.parent_table(ens.NTU_BONE_PAIRS, 25)
    assert ntu[20] == 20 and ntu[0] == 1      # spine is the NTU root; joint 1 -> 2 (1-indexed)
    with pytest.raises(ValueError):
        ens.parent_table(ens.MEDIAPIPE_BONE_PAIRS[:-1], 33)


def test_derive_modalities_bit_exact(golden):
    fx = golden("ensemble_fixtures.npz")
    pairs = [tuple(p) for p in fx["bone_pairs"]]
    got = eo.derive_modalities(fx["mod_input"], pairs)
    for s in STREAMS:
        assert np.array_equal(got[s], fx[f"mod_{s}"]), s
    # the batched form equals the per-window form
    batch = np.stack([fx["mod_input"], 2 * fx["mod_input"]])
    gb = eo.derive_modalities(batch, pairs)
    for s in STREAMS:
        assert np.array_equal(gb[s][0], fx[f"mod_{s}"]), s


def test_ensemble_scores_match_reference(golden):
    fx = golden("ensemble_fixtures.npz")
    pairs = [tuple(p) for p in fx["bone_pairs"]]
    models = oracle_models()
    scores, fused = eo.run_ensemble_inference(list(fx["ens_windows"]), models,
                                              tuple(fx["weights"]), pairs)
    assert np.abs(scores - fx["ens_scores"]).max() < 1e-6
    for s in STREAMS:
        with torch.no_grad():
            got = np.stack([models[s](torch.from_numpy(
                eo.derive_modalities(w, pairs)[s]).unsqueeze(0)).numpy()[0]
                for w in fx["ens_windows"]])
        assert np.abs(got - fx[f"ens_logits_{s}"]).max() < 1e-5, s
