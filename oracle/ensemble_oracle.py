"""CPU restatement of the 4-stream ensemble inference (TEST INFRASTRUCTURE ONLY).

* :func:`derive_modalities` <- ``inference_pipeline.py:284-309`` (one window, numpy fp32:
  bone = joint - joint[parent] per BONE_PAIRS, motion = x[t+1] - x[t], last frame 0);
  also the batch form of ``data_gen/gen_bone_data*.py`` / ``gen_motion_data*.py``.
* :func:`run_ensemble_inference` <- ``inference_pipeline.py:342-370`` (per window, per
  stream: batch-1 eval forward, ``ensemble_logits += alpha * logits`` in a float64
  accumulator, max-shifted softmax, score = class 1).

Pinned against the reference's own ``derive_modalities`` / ``run_ensemble_inference``
(imported with cv2/mediapipe stubbed, ``tests/golden/gen_ensemble_fixtures.py``) by
``tests/test_oracle_ensemble.py``.
"""
from __future__ import annotations

import numpy as np
import torch

MODALITIES = ("joint", "bone", "joint_motion", "bone_motion")


def derive_modalities(joint, bone_pairs):
    """joint: (C, T, V, M) or (N, C, T, V, M) float32 -> dict of the four streams."""
    j = np.asarray(joint, dtype=np.float32)
    bone = np.zeros_like(j)
    for v, p in bone_pairs:
        bone[..., v, :] = j[..., v, :] - j[..., p, :]
    T = j.shape[-3]

    def motion(a):
        out = np.zeros_like(a)
        out[..., :T - 1, :, :] = a[..., 1:, :, :] - a[..., :T - 1, :, :]
        return out

    return {"joint": j, "bone": bone, "joint_motion": motion(j), "bone_motion": motion(bone)}


def run_ensemble_inference(windows, models, weights, bone_pairs):
    """windows: iterable of (C, T, V, M) arrays; models: dict stream -> eval-mode CPU Model.
    Returns (scores (W,), fused float64 logits (W, num_class))."""
    scores, fused = [], []
    with torch.no_grad():
        for w in windows:
            mods = derive_modalities(w, bone_pairs)
            acc = None
            for name, alpha in zip(MODALITIES, weights):
                x = torch.from_numpy(mods[name]).unsqueeze(0).float()
                logits = models[name](x).numpy()[0]
                term = (np.float32(alpha) * logits).astype(np.float64)
                acc = term if acc is None else acc + term
            e = np.exp(acc - acc.max())
            scores.append(float(e[1] / e.sum()))
            fused.append(acc)
    return np.array(scores), np.stack(fused)
