"""mivs.neighbors — the ``cuvs.neighbors`` modules the reference imports (ivf_flat, brute_force).

``ivf_pq`` and ``cagra`` are named by the reference (index_building_coordinator.py:398-414) but are
outside this round's hot path; importing them raises a clear error.
"""
from . import brute_force, ivf_flat  # noqa: F401

__all__ = ["ivf_flat", "brute_force"]
