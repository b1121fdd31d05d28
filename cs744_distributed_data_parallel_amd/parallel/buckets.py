"""Gradient bucket planning.

Reference behaviour being replaced: torch DDP's Reducer (``/root/reference/src/Part 3/main.py:61``)
buckets parameters in reverse registration order with a 25 MiB cap (1 MiB first bucket), and after
iteration 1 rebuilds the buckets in the observed gradient-ready order. For VGG-11 that yields
9.46 MB / 27.16 MB / 0.31 MB buckets.

MI355X choice: xGMI is point-to-point (7 links x ~153 GB/s per GPU) and a ring all-reduce is
per-link bound, so a 27 MB bucket that only becomes ready late in backward serialises behind the
remaining compute. The default cap here is smaller (8 MiB; first bucket 1 MiB) so the large
late-layer gradients (VGG-11's 9.4 MB conv weights) each launch as soon as they are ready and
overlap the rest of backward, while staying large enough for RCCL to reach bandwidth.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

DEFAULT_BUCKET_CAP_MB = 8.0
DEFAULT_FIRST_BUCKET_CAP_MB = 1.0


def plan_buckets(
    nbytes_in_launch_order: Sequence[int],
    cap_mb: float = DEFAULT_BUCKET_CAP_MB,
    first_cap_mb: float = DEFAULT_FIRST_BUCKET_CAP_MB,
) -> List[List[int]]:
    """Greedy bucketing. Returns lists of positions (into the launch-ordered sequence).

    A bucket closes as soon as it reaches its cap (a single tensor larger than the cap gets a bucket
    of its own), exactly like torch's ``compute_bucket_assignment_by_size``.
    """
    cap = int(cap_mb * 1024 * 1024)
    first = int(first_cap_mb * 1024 * 1024)
    buckets: List[List[int]] = []
    cur: List[int] = []
    size = 0
    limit = first if first > 0 else cap
    for i, nb in enumerate(nbytes_in_launch_order):
        cur.append(i)
        size += int(nb)
        if size >= limit:
            buckets.append(cur)
            cur, size = [], 0
            limit = cap
    if cur:
        buckets.append(cur)
    return buckets


def contiguous_bucket_starts(n_params: int, buckets_over_reversed: List[List[int]]) -> List[int]:
    """For an arena in *model order* and buckets planned over the *reversed* order, return the
    ``bucket_starts`` boundaries expected by the reducer (bucket b covers arena indices
    [starts[b+1], starts[b]) -- descending ranges)."""
    starts = [n_params]
    for b in buckets_over_reversed:
        starts.append(n_params - 1 - b[-1])
    return starts


def bucket_ranges_in_arena(offsets: Sequence[int], aligned_numels: Sequence[int], starts: Sequence[int]) -> List[Tuple[int, int]]:
    """Flat element ranges of each bucket, given parameter offsets in the arena."""
    ranges = []
    for b in range(len(starts) - 1):
        lo, hi = sorted((starts[b], starts[b + 1]))
        s = offsets[lo]
        e = offsets[hi - 1] + aligned_numels[hi - 1]
        ranges.append((s, e))
    return ranges
