"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the DlQuantization hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package. ``aimet_amd`` (the product) never does.

* :mod:`oracle.oracle` -- ctypes face of ``liboracle.so`` (``dlq_oracle.c``: C restatement
  of the reference CPU arithmetic, pinned by ``tests/golden``).
* :mod:`oracle.ref` -- ctypes face of ``_ref/libdlq_ref.so`` (the reference C++ compiled
  in place from ``/root/reference``; only present in the build container).
* :mod:`oracle.torch_ref` -- float32 torch/numpy restatements of the reference's Python-side
  arithmetic (STE mask, learned-grid, AdaRound soft rounding).
"""
