"""ORACLE — test infrastructure only.

This package is the CPU checker for the MI355X two-tower training step.  It is a
from-scratch fp32 PyTorch-CPU restatement of the reference's hot path
(DiegoPaniagua23/music-recommendation-multimodal, ``src/models`` + the
``src/train.py`` InfoNCE step), pinned against golden fixtures that were produced by
running the reference's own modules in the survey container (``tools/make_golden.py``
-> ``tests/golden/*.npz``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything from here, and only as the checker / the timed CPU baseline.  The
product path (``music-recommendation-multimodal_amd``) never imports it and fails loudly
when its HIP library is missing.
"""
