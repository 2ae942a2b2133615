"""Multi-GPU hash-partitioned group-by (one process per GPU, RCCL all-to-all).

Implemented in polaroid_amd/distributed.py once the partial-state C-ABI lands.
"""

from __future__ import annotations


def group_by_agg(df, key, aggs, predicate=None, info=None):  # pragma: no cover - placeholder
    raise NotImplementedError("multi-GPU group-by is not wired yet")
