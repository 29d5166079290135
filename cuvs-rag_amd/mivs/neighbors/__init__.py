"""mivs.neighbors — the ``cuvs.neighbors`` modules the reference imports (ivf_flat, ivf_pq, brute_force),
plus ``refine`` (exact re-ranking of candidates) and ``streaming.search_host`` (host queries with overlapped copies).

``cagra`` is named by the reference (index_building_coordinator.py:405-412) but is outside the
hot path.
"""
from . import brute_force, ivf_flat, ivf_pq, streaming  # noqa: F401
from .refine import refine  # noqa: F401

__all__ = ["ivf_flat", "ivf_pq", "brute_force", "streaming", "refine"]
