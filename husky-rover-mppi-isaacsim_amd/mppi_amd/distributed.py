"""K-sharded MPPI step over torch.distributed (RCCL on MI355X), one process per GPU.

SURVEY.md §8(e).  Trajectories are independent until the softmax, so rank g
owns a contiguous, leaf-aligned slice of the K samples (Philox is keyed by the
GLOBAL trajectory index, so every rank draws exactly the noise the single-GPU
step would).  Per step each rank reduces its slice to one record
[m, S, V1[H], V2[H]] (float64, 2H+2 values), the ranks all-gather the records
(one collective, ~1.6 KB per rank at H=100) and every rank combines them in
rank order and runs the optimal rollout itself — identical outputs on all
ranks, no broadcast.  When every shard holds a power-of-two number of 256-wide
leaves (e.g. 65536 per GPU) the result is bitwise identical to the one-GPU step.

The reference has no multi-GPU path; this is the MI355X extension of
MPPI_isaac.py:505-720.
"""
from __future__ import annotations

LEAF = 256   # trajectories per reduction leaf (csrc/mppi_kernels.hip leaf_records)


def shard_bounds(K: int, world: int):
    """[(begin, count)] per rank: contiguous, leaf-aligned except the last shard."""
    if world <= 1:
        return [(0, K)]
    leaves = (K + LEAF - 1) // LEAF
    per = (leaves + world - 1) // world
    out = []
    for g in range(world):
        b = min(K, g * per * LEAF)
        e = min(K, (g + 1) * per * LEAF)
        out.append((b, e - b))
    return out


def exchange_records(record, gathered, group=None):
    """All-gather this rank's record into ``gathered`` (world * E doubles, rank order).

    RCCL/NCCL: one all_gather_into_tensor.  gloo (CPU tests): all_gather into views.
    """
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(gathered, record, group=group)
    else:
        world = dist.get_world_size(group)
        E = record.numel()
        dist.all_gather([gathered[i * E:(i + 1) * E] for i in range(world)], record, group=group)
    return gathered


class ShardedMPPI:
    """One rank of a K-sharded controller: this rank's engine + the record exchange.

    ``params_kw`` are make_params keywords (dt, temperature, seed, ...); the
    shard's size and global offset come from shard_bounds(K_global, world).
    The engine runs on a dedicated torch stream that RCCL also uses, so the
    partial kernel, the all-gather and the finish kernel are stream-ordered
    with no host synchronisation in between.
    """

    def __init__(self, K_global: int, H: int, device, group=None, engine_factory=None, always_exchange=False,
                 **params_kw):
        """``engine_factory(K, H, k_offset, device)`` replaces the HIP engine (CPU protocol tests
        drive the same exchange with an oracle-backed stand-in); ``device="cpu"`` then skips the
        HIP stream and keeps the exchange buffers in host memory (gloo).  ``always_exchange``
        runs the partial step, the collective and the finish even at world size 1 (tests of the
        RCCL path on a one-GPU host)."""
        self.always_exchange = bool(always_exchange)
        import contextlib

        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.K_global = int(K_global)
        self.H = int(H)
        self.k_begin, self.k_count = shard_bounds(self.K_global, self.world)[self.rank]
        # a rank left without trajectories (K < world * LEAF) still takes part in every exchange:
        # it contributes the empty record (m = +inf, S = V = 0), which the combine tree passes
        # through, and runs the finish like every other rank.  Its engine only serves the finish.
        self.empty = self.k_count <= 0
        k_eng = LEAF if self.empty else self.k_count
        k_off = min(self.k_begin, self.K_global)
        if engine_factory is None:
            from . import _lib
            self.engine = _lib.Engine(_lib.make_params(k_eng, H, k_offset=k_off, **params_kw), device)
        else:
            self.engine = engine_factory(k_eng, H, k_off, device)
        if device == "cpu":
            self.stream = None
            self._ctx = contextlib.nullcontext
            tdev = "cpu"
        else:
            self.stream = torch.cuda.Stream(device=device)
            self.engine.set_stream(self.stream.cuda_stream)
            self._ctx = lambda: torch.cuda.stream(self.stream)
            tdev = f"cuda:{device}"
        E = self.engine.record_len()
        self.record = torch.empty(E, dtype=torch.float64, device=tdev)
        self.gathered = torch.empty(self.world * E, dtype=torch.float64, device=tdev)

    def step(self, proj="3d", step=0, copy=True):
        """One MPPI_step over K_global trajectories; outputs (identical on all ranks) in host memory."""
        with self._ctx():
            if self.world == 1 and not self.always_exchange:
                return self.engine.step(proj, step, copy)
            if self.empty:
                self.record.zero_()
                self.record[0] = float("inf")
            else:
                self.engine.step_partial(self.record.data_ptr(), proj, step)
            exchange_records(self.record, self.gathered, self.group)
            return self.engine.step_finish(self.gathered.data_ptr(), self.world, copy)

    def close(self):
        self.engine.close()
