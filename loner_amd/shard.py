"""Data-parallel sharding of a window's ray batch.

Rays are independent given the parameters, so a step shards by rays: rank r renders the
contiguous slice ``shard_range(R, r, world)`` of the concatenated window batch (the reference
concatenates keyframes in window order, optimizer.py:417-424, so contiguous slices give every rank
whole keyframes).  Three things make the per-rank results sum to the single-GPU step:

  * draws are keyed by the GLOBAL ray index (``StepEngine(ray_offset=start)``);
  * the loss normalisers are global: the opaque-ray count is all-reduced before the loss
    (optimizer.py:752-753,841-842 average over opaque rays) and the LOS mean uses the global
    rays x samples (:833-834); ray 0's far bound (the :724 broadcast) is the GLOBAL ray 0's;
  * one all-reduce(SUM) of the flat gradient before the (identical) Adam on every rank, and of
    the OGM gradient before its SGD step.
"""


def shard_range(n_rays: int, rank: int, world: int):
    """[start, end) of rank's contiguous share; shares differ by at most one ray."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(n_rays, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)
