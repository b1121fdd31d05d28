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

That fixed-cap plan is only the fallback (and what an explicit ``bucket_cap_mb`` gets). By default
the reducer *designs* its plan after the first iteration (:func:`plan_buckets_timed`): it knows when
each gradient became ready on the GPU in that iteration (events recorded by per-parameter hooks)
and what a collective of S bytes costs on this communicator (``alpha + beta * S``, fitted from a
few all-reduces at rebuild time), and it picks the contiguous partition of the ready-ordered
gradients whose last all-reduce finishes first. The comm stream runs one bucket at a time, so a
bucket starts at max(its last gradient's ready time, the previous bucket's end): too many buckets
pay alpha (RCCL's per-collective latency, several us on xGMI) over and over, too few start late or
leave a large tail exposed after backward. The plan therefore depends on the batch per GPU (the
backward timeline), the world size and the links (alpha, beta) -- e.g. at the reference's
strong-scaling point (32 images per GPU at W = 8) backward is only ~0.3 ms and the planner keeps the
tail bucket (the first layers, ready last) small; at 256 images per GPU it can afford fewer buckets.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

DEFAULT_BUCKET_CAP_MB = 8.0
DEFAULT_FIRST_BUCKET_CAP_MB = 1.0


def plan_buckets_timed(
    nbytes_in_launch_order: Sequence[int],
    ready_s: Sequence[float],
    alpha_s: float,
    beta_s_per_byte: float,
    bucket_penalty_s: float = 3e-6,
) -> Tuple[List[List[int]], dict]:
    """Bucket plan that minimises the modelled end of the last all-reduce plus a small cost per
    bucket (exact DP over Pareto fronts of (end, bucket count), O(n^2 * front)).

    ``ready_s[i]``: when gradient i (launch order) is ready, seconds from any common origin;
    a collective of S bytes takes ``alpha_s + beta_s_per_byte * S`` on the comm stream and
    collectives run one after another. ``bucket_penalty_s`` prices what the end time does not see:
    every collective is a kernel whose workgroups take CUs from the backward GEMMs (and one more
    launch), so among plans that end (nearly) together the one with fewer buckets wins.
    Returns (groups of launch positions, model summary).
    """
    n = len(nbytes_in_launch_order)
    if n == 0:
        return [], {}
    ready = []
    m = float("-inf")
    for r in ready_s:  # a bucket cannot launch before every gradient it holds (monotone)
        m = max(m, float(r))
        ready.append(m)
    pre = [0]
    for b in nbytes_in_launch_order:
        pre.append(pre[-1] + int(b))
    # front[j]: non-dominated (end, count, i, index into front[i]) for the prefix [0, j)
    front: List[List[Tuple[float, int, int, int]]] = [[] for _ in range(n + 1)]
    front[0] = [(float("-inf"), 0, -1, -1)]
    for j in range(1, n + 1):
        cand = []
        for i in range(j):
            dur = alpha_s + beta_s_per_byte * (pre[j] - pre[i])
            for k, (e, c, _, _) in enumerate(front[i]):
                cand.append((max(e, ready[j - 1]) + dur, c + 1, i, k))
        cand.sort(key=lambda t: (t[1], t[0]))  # by count, then end
        keep = []
        for t in cand:
            if keep and t[1] == keep[-1][1]:
                continue  # same count: the earliest end is already kept
            if keep and t[0] >= keep[-1][0] - 1e-12:
                continue  # more buckets but no earlier end: dominated
            keep.append(t)
        front[j] = keep
    best = min(front[n], key=lambda t: t[0] + bucket_penalty_s * t[1])
    groups = []
    j, t = n, best
    while j > 0:
        _, _, i, k = t
        groups.append(list(range(i, j)))
        j, t = i, front[i][k] if i > 0 else None
    groups.reverse()
    info = {
        "backward_end_us": round((ready[-1] - ready[0]) * 1e6, 2),
        "comm_end_us": round((best[0] - ready[0]) * 1e6, 2),
        "exposed_us": round(max(0.0, best[0] - ready[-1]) * 1e6, 2),
        "alpha_us": round(alpha_s * 1e6, 3),
        "algbw_GBps": round(1.0 / beta_s_per_byte / 1e9, 2) if beta_s_per_byte > 0 else None,
    }
    return groups, info


def fit_comm_model(sizes_bytes: Sequence[int], times_s: Sequence[float]) -> Tuple[float, float]:
    """Least-squares ``t = alpha + beta * S`` over measured all-reduce times (alpha, beta >= 0)."""
    n = len(sizes_bytes)
    sx = sum(sizes_bytes)
    sy = sum(times_s)
    sxx = sum(x * x for x in sizes_bytes)
    sxy = sum(x * y for x, y in zip(sizes_bytes, times_s))
    den = n * sxx - sx * sx
    if n < 2 or den <= 0:
        return max(0.0, sy / max(n, 1)), 0.0
    beta = (n * sxy - sx * sy) / den
    alpha = (sy - beta * sx) / n
    return max(alpha, 0.0), max(beta, 0.0)


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
