"""koordinator_amd — MI355X-native evaluator for koord-scheduler's per-pod sweep.

The product is ``libkoordgpu.so`` (HIP kernels for gfx950 behind the C ABI in
``include/koordgpu.h``).  This Python package is the host-side mirror used by
tests and the benchmark: ctypes bindings (:mod:`.abi`, :mod:`.runtime`), the
plugin-args mirror with the reference's defaults (:mod:`.config`), the
snapshot → structure-of-arrays ingestion (:mod:`.cluster`) and the synthetic
cluster generators C1–C5 (:mod:`.synth`).
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
