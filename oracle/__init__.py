"""CPU oracle for the Shift-GCN hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / reported CPU baseline. The product path
(``shift-gcn_amd/shiftgcn``) never imports it and fails loudly without its HIP library.

* :mod:`oracle.shift_oracle` — vectorised numpy restatement of the reference CUDA
  temporal-shift extension (``model/Temporal_shift/cuda/shift_cuda_kernel.cu``).
* :mod:`oracle.shift_loops`  — scalar-loop restatement used to pin the vectorised one.
* :mod:`oracle.model_oracle` — PyTorch-eager CPU restatement of ``model/shift_gcn.py``
  (``tcn``, ``Shift_tcn``, ``Shift_gcn``, ``TCN_GCN_unit``, ``Model``) on top of the
  numpy shift, plus the reference training-step semantics (``main.py``).

Pinning: see each module's header and DESIGN.md §Oracle.
"""
