"""Golden fixtures for the 4-stream ensemble (BASELINE config 4), made by running the
REFERENCE's own ``derive_modalities`` and ``run_ensemble_inference``
(``inference_pipeline.py:284-370``) on CPU. Run only where ``/root/reference`` exists:

    python tests/golden/gen_ensemble_fixtures.py

``inference_pipeline.py`` imports cv2 and mediapipe at module level (used only by its
video front end, not by the two functions called here); both are absent from this image
and are replaced by empty module objects. ``Tensor.cuda`` is the identity during the run
(no GPU here). The four stream models are the reference ``Model`` (MediaPipe, 33 joints,
1 person, 2 classes) with deterministic formula weights; the shift extension is the numpy
restatement, exactly as in ``gen_fixtures.py``. Only outputs are stored.

Output: ``tests/golden/ensemble_fixtures.npz``.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import formula  # noqa: E402
import gen_fixtures as gf  # noqa: E402

REF = gf.REF
STREAMS = ("joint", "bone", "joint_motion", "bone_motion")
ENS_T = 64          # window length of the fused-score fixture (any T runs the model)
MOD_T = 40          # window length of the modality fixture


def window(seed, T, V=33, M=1):
    return formula.tensor((3, T, V, M), seed, 1.0).numpy()


def main():
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    ref_sg, _ = gf._import_reference()
    for name in ("cv2", "mediapipe"):
        sys.modules.setdefault(name, types.ModuleType(name))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import inference_pipeline as ip  # noqa: E402

    out = {}
    w = window(501, MOD_T)
    mods = ip.derive_modalities(w)
    out["mod_input"] = w
    for k in STREAMS:
        out[f"mod_{k}"] = mods[k]
    out["bone_pairs"] = np.array(ip.BONE_PAIRS, dtype=np.int64)
    out["weights"] = np.array(ip.ENSEMBLE_WEIGHTS_DEFAULT, dtype=np.float64)

    graph_mod = types.ModuleType("fixture_graph")

    class Graph:
        def __init__(self, **kw):
            self.A = np.zeros((3, 1, 1))

    graph_mod.Graph = Graph
    sys.modules["fixture_graph"] = graph_mod
    models = {}
    for k, s in enumerate(STREAMS):
        with gf._cpu_construction():
            m = ref_sg.Model(num_class=2, num_point=33, num_person=1,
                             graph="fixture_graph.Graph")
        formula.fill_state(m, seed=701 + 13 * k)
        models[s] = m.eval()
    wins = [window(601 + i, ENS_T) for i in range(3)]
    # one zero-padded tail window as create_sliding_windows makes (inference_pipeline.py:272-276)
    wins[2][:, ENS_T // 2:] = 0.0
    windows = [(x, 0, ENS_T, ENS_T) for x in wins]
    cuda0 = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        res = ip.run_ensemble_inference(windows, models, ip.ENSEMBLE_WEIGHTS_DEFAULT)
    finally:
        torch.Tensor.cuda = cuda0
    out["ens_windows"] = np.stack(wins)
    out["ens_scores"] = np.array([r[0] for r in res], dtype=np.float64)
    with torch.no_grad():
        for s in STREAMS:
            out[f"ens_logits_{s}"] = np.stack([
                models[s](torch.from_numpy(ip.derive_modalities(x)[s]).unsqueeze(0)).numpy()[0]
                for x in wins])
    path = os.path.join(HERE, "ensemble_fixtures.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
