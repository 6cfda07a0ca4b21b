"""Multi-GPU replication (new in this build; the reference is shared-memory
Hogwild only, src/model/LINE.cpp:162).

One process per GPU.  Every rank holds the whole graph and both embedding
tables, runs its own disjoint range of global sample indices (Hogwild inside
the GPU), and the ranks exchange what they learned through the snapshot-delta
rule

    delta_r = T_r - T_snap ;  all_reduce(delta, SUM) over RCCL (xGMI)
    T = T_snap + sum_r delta_r      (or the mean, --sync mean)

With sum, every sample's update lands on every replica exactly once -- the
multi-GPU analogue of the reference's single shared table.  Added one
exchange late, though, a hub row's summed deltas (thousands of updates per
exchange on every rank, each computed against the stale row) overshoot, and
training diverges at 4 and 8 ranks (tools/replica_sim.py).  The
adaptive rule (the default) scales row i's summed delta by
    s_i + (1 - s_i) / N,   s_i = min(1, c0 / k_i),
k_i = the row's expected updates per exchange over all ranks (sampler
marginals x samples per exchange x N): the sum for rows updated a few times
per exchange, the mean for the hubs.

Two schedules:
  DeltaAllReduce  synchronous: the collective runs between two steps.
  OverlapSync     one exchange late: begin() snapshots this rank's delta and
                  starts its all-reduce asynchronously (ProcessGroupNCCL runs it
                  on its own stream, ordered after the compute stream's current
                  point), the next training step runs meanwhile, and end()
                  makes the compute stream wait for it and folds the other
                  ranks' deltas in.  ReplicaSync = OverlapSync over a ProNet
                  context's device tables with the fused HIP passes of
                  replica_sync.hip.
"""
import torch
import torch.distributed as dist


class _DeviceArray:
    """Zero-copy view of a libsmore_hip table for torch.as_tensor."""

    def __init__(self, ptr, shape):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "<f4", "data": (int(ptr), False),
                                         "version": 2, "strides": None}


def table_tensor(pn, which):
    ptr, stride = pn.table_device(which)
    t = torch.as_tensor(_DeviceArray(ptr, (pn.MAX_vid, stride)), device="cuda")
    if t.data_ptr() != ptr:
        raise RuntimeError("table view is not zero-copy")
    return t


def hub_slots_tensor(pn):
    """Zero-copy view of the C table's hub slot rows V .. V + H of the block
    setup (blocks.cpp), or None without hubs."""
    H, first, _, _ = pn.block_hubs()
    if not H:
        return None
    ptr, stride = pn.table_device(1)
    p = ptr + first * stride * 4
    t = torch.as_tensor(_DeviceArray(p, (H, stride)), device="cuda")
    if t.data_ptr() != p:
        raise RuntimeError("slot view is not zero-copy")
    return t


def block_hubs(pn, samples_per_exchange, c0=2048.0):
    """BlockSync's `hubs` argument for a ProNet context after block_setup
    (None without hubs): its slot view, the adaptive scales for
    `samples_per_exchange` samples per rank per sub-round, the fused HIP
    passes, and the context's slot load / store."""
    slots = hub_slots_tensor(pn)
    if slots is None:
        return None
    scale = torch.from_numpy(pn.block_hub_scales(samples_per_exchange, c0)).to(slots.device)
    return {"slots": slots, "scale": scale, "passes": HipPasses(pn), "load": pn.block_hubs_load,
            "store": pn.block_hubs_store}


class DeltaAllReduce:
    """Synchronous snapshot-delta exchange over same-shaped tensors on every rank."""

    def __init__(self, tensors, mean=False, group=None):
        self.tensors = list(tensors)
        self.snaps = [t.clone() for t in self.tensors]
        self.mean = mean
        self.group = group

    def allreduce(self):
        world = dist.get_world_size(self.group)
        for t, s in zip(self.tensors, self.snaps):
            t.sub_(s)                                        # t := local delta
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            if self.mean:
                t.div_(world)
            t.add_(s)                                        # t := snap + sum of deltas
            s.copy_(t)


class TorchPasses:
    """The exchange passes as torch ops (CPU tensors in the gloo tests)."""

    @staticmethod
    def begin(T, S, D, R):
        torch.sub(T, S, out=D)
        R.copy_(D)
        S.copy_(T)

    @staticmethod
    def end(T, S, D, R, scale):
        if torch.is_tensor(scale):          # per-row scale (adaptive rule)
            scale = scale.view(-1, *([1] * (R.dim() - 1)))
        R.mul_(scale).sub_(D)
        T.add_(R)
        S.add_(R)

    @classmethod
    def cycle(cls, T, S, D, R, scale):
        cls.end(T, S, D, R, scale)
        cls.begin(T, S, D, R)


class HipPasses:
    """The same passes as one fused HIP kernel each (replica_sync.hip), on the
    context stream."""

    def __init__(self, pn):
        self.pn = pn

    def begin(self, T, S, D, R):
        self.pn.delta_begin(T.data_ptr(), S.data_ptr(), D.data_ptr(), R.data_ptr(), T.numel())

    def end(self, T, S, D, R, scale):
        if torch.is_tensor(scale):
            self.pn.delta_end_rows(T.data_ptr(), S.data_ptr(), D.data_ptr(), R.data_ptr(), scale.data_ptr(),
                                   T.shape[0], T.shape[1])
        else:
            self.pn.delta_end(T.data_ptr(), S.data_ptr(), D.data_ptr(), R.data_ptr(), scale, T.numel())

    def cycle(self, T, S, D, R, scale):
        if torch.is_tensor(scale):
            self.pn.delta_cycle_rows(T.data_ptr(), S.data_ptr(), D.data_ptr(), R.data_ptr(), scale.data_ptr(),
                                     T.shape[0], T.shape[1])
        else:
            self.pn.delta_cycle(T.data_ptr(), S.data_ptr(), D.data_ptr(), R.data_ptr(), scale, T.numel())


class OverlapSync:
    """One-exchange-late snapshot-delta exchange whose collective overlaps the
    next compute step (see the module docstring).

        begin():  [end() of the previous exchange, fused with this begin];
                  D = T - S; R = D; S = T; all_reduce(R) started asynchronously
        end():    wait for the collective; X = scale*R - D; T += X; S += X

    After end() every replica holds every rank's updates up to the matching
    begin(), plus its own since."""

    def __init__(self, tensors, mean=False, group=None, passes=None, hot_idx=None, row_scale=None):
        self.T = list(tensors)
        self.S = [t.clone() for t in self.T]
        self.D = [torch.zeros_like(t) for t in self.T]
        self.R = [torch.zeros_like(t) for t in self.T]
        self.mean = mean
        self.group = group
        self.passes = passes or TorchPasses()
        self.works = None
        # adaptive rule: one per-row scale tensor per table (replaces `mean`)
        self.row_scale = list(row_scale) if row_scale is not None else None
        # hub rows (one int64 index tensor per table) exchanged by hot(); sum only
        self.hot_idx = [] if (mean or row_scale is not None or not hot_idx) else list(hot_idx)

    def hot(self):
        """Synchronous exchange of the hub rows between two training launches:
        D' = T_h - S_h;  R' = all_reduce(D');  T_h += R' - D';  S_h += R'.
        Between a begin() and its end() S holds the rank's own snapshot, so D'
        is the change since then and the pending end() adds only the older
        deltas: every update still lands once on every replica."""
        for T, S, idx in zip(self.T, self.S, self.hot_idx):
            D = T.index_select(0, idx) - S.index_select(0, idx)
            R = D.clone()
            dist.all_reduce(R, op=dist.ReduceOp.SUM, group=self.group)
            T.index_add_(0, idx, R - D)
            S.index_add_(0, idx, R)

    def begin(self):
        if self.works is not None:      # fold the previous exchange in and start this one: one pass
            for w in self.works:
                w.wait()
            for i, (T, S, D, R) in enumerate(zip(self.T, self.S, self.D, self.R)):
                self.passes.cycle(T, S, D, R, self._scale(i))
        else:
            for T, S, D, R in zip(self.T, self.S, self.D, self.R):
                self.passes.begin(T, S, D, R)
        self.works = [dist.all_reduce(R, op=dist.ReduceOp.SUM, group=self.group, async_op=True) for R in self.R]

    def _scale(self, i=0):
        if self.row_scale is not None:
            return self.row_scale[i]
        return 1.0 / dist.get_world_size(self.group) if self.mean else 1.0

    def end(self):
        if self.works is None:
            return
        for w in self.works:
            w.wait()
        for i, (T, S, D, R) in enumerate(zip(self.T, self.S, self.D, self.R)):
            self.passes.end(T, S, D, R, self._scale(i))
        self.works = None

    def allreduce(self):
        """Synchronous use: begin() then end()."""
        self.begin()
        self.end()


def adaptive_scale(rate, updates, world, c0=64.0):
    """Per-row scale of the adaptive rule: rate = expected touches per sample
    of each row, `updates` samples per rank per exchange (float32 numpy)."""
    import numpy as np
    k = np.asarray(rate, np.float64) * float(updates) * world
    s = np.minimum(1.0, c0 / np.maximum(k, 1e-300))
    return (s + (1.0 - s) / world).astype(np.float32)


class BlockSync:
    """The 2-D block schedule over torch.distributed (one process per GPU;
    the group driver's twin is exchange.cpp group_block_*).

    Rank r owns the W rows of part r; the C rows are cut into nb = 2N blocks
    (`c_bounds`, nb + 1 row bounds).  Sub-round s (counted over the whole run)
    trains cell (r, (2r + s) mod nb) -- `train(block)` queues it on the current
    stream -- then sends that C block to rank r - 1 and receives block
    (2r + s + 2) mod nb from rank r + 1, asynchronously (NCCL: on its own
    stream, ordered after the cell); the cell of sub-round s + 2 waits for that
    receive, so a transfer overlaps one whole sub-round.  No row trains on two
    ranks at once: nothing is all-reduced.  finish() drains the transfers and,
    with gather=True, gives every rank every W part (from its owner) and every
    C block (from its holder).

    W, C: the table tensors (rows x stride; CPU tensors in the gloo tests).
    Over gloo, CUDA blocks are staged through host memory (gloo's send/recv
    take CPU tensors).

    hubs (LINE-2 hub C rows, blocks.cpp): a dict with `slots` (this rank's
    copy of the H hub rows, a view of C's slot rows), `scale` (per-slot
    exchange scales), optional `passes` (HipPasses / TorchPasses), `load` and
    `store` (slots <- hub rows / hub rows <- slots).  Every cell trains the
    slots; after each sub-round their deltas are all-reduced one late
    (OverlapSync, adaptive per-slot scales) ahead of the rotation; finish()
    folds the last exchange in (every rank's slots equal) and, with
    gather=True, stores the slots into the hub rows before the gather."""

    def __init__(self, W, C, w_bounds, c_bounds, group=None, hubs=None):
        self.W, self.C = W, C
        self.wb = [int(x) for x in w_bounds]
        self.cb = [int(x) for x in c_bounds]
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.nb = len(self.cb) - 1
        if self.nb != 2 * self.world or len(self.wb) != self.world + 1:
            raise ValueError("block schedule: N + 1 W bounds and 2N + 1 C bounds for N ranks")
        self.ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.world))
        self.staged = dist.get_backend(group) == "gloo" and C.is_cuda
        self.s = 0                 # sub-rounds done
        self.pending = [None, None]   # (works, post) of the last two rotations, by sub-round parity
        self.hubs = hubs
        self.hub_sync = None
        if hubs is not None:
            if hubs.get("load") is not None:
                hubs["load"]()        # slots <- hub rows, on the current stream
            self.hub_sync = OverlapSync([hubs["slots"]], group=group, passes=hubs.get("passes"),
                                        row_scale=[hubs["scale"]])

    def block(self, s=None):
        """The C block this rank trains at sub-round s (default: the next)."""
        s = self.s if s is None else s
        return (2 * self.rank + s) % self.nb

    def rows(self, b):
        return self.C[self.cb[b]:self.cb[b + 1]]

    def _wait(self, slot):
        p = self.pending[slot]
        if p is not None:
            works, post = p
            for w in works:
                w.wait()
            if post is not None:
                post()
            self.pending[slot] = None

    def sub_round(self, train, parts=1):
        """Train this rank's cell of the next sub-round and start its rotation.
        parts > 1: the cell in `parts` launches, train(block, q) for q in
        range(parts), the hub slots exchanged after each (blocks.cpp
        cell_launches)."""
        s = self.s
        self._wait(s & 1)               # the block received at sub-round s - 2
        b = self.block(s)
        for q in range(parts):
            if parts == 1:
                train(b)
            else:
                train(b, q)
            if self.hub_sync is not None:
                self.hub_sync.begin()   # the hub slots' deltas, one late, ahead of the rotation
        send, recv = self.rows(b), self.rows((b + 2) % self.nb)
        dst = self.ranks[(self.rank - 1) % self.world]
        src = self.ranks[(self.rank + 1) % self.world]
        post = None
        if self.staged:
            send_h = send.cpu()
            recv_h = torch.empty_like(recv, device="cpu")
            ops = [dist.P2POp(dist.isend, send_h, dst, self.group), dist.P2POp(dist.irecv, recv_h, src, self.group)]

            def post(recv=recv, recv_h=recv_h):
                recv.copy_(recv_h)
        else:
            ops = [dist.P2POp(dist.isend, send, dst, self.group), dist.P2POp(dist.irecv, recv, src, self.group)]
        self.pending[s & 1] = (dist.batch_isend_irecv(ops), post)
        self.s += 1

    def epoch(self, train, parts=1):
        """nb sub-rounds: every cell of this rank's W part once."""
        for _ in range(self.nb):
            self.sub_round(train, parts)

    def holder(self, b):
        """The rank holding C block b's latest rows once the transfers drained."""
        return ((b - self.s) % self.nb) // 2

    def finish(self, gather=True):
        self._wait(0)
        self._wait(1)
        if self.hub_sync is not None:
            self.hub_sync.end()         # every rank's slots equal
            if gather and self.hubs.get("store") is not None:
                self.hubs["store"]()    # hub rows <- slots, before the blocks are gathered
        if not gather:
            return
        for p in range(self.world):
            if self.wb[p + 1] > self.wb[p]:
                dist.broadcast(self.W[self.wb[p]:self.wb[p + 1]], src=self.ranks[p], group=self.group)
        for b in range(self.nb):
            dist.broadcast(self.rows(b), src=self.ranks[self.holder(b)], group=self.group)


class ReplicaSync(OverlapSync):
    """OverlapSync over a ProNet context's device tables (W and C), with the
    fused HIP passes; the context runs on torch's current stream so the
    passes, the training kernels and the collective are ordered on it.

    sync: "adaptive" (default; needs `updates`, the samples each rank trains
    per exchange, and `model`/`K` for the row rates), "mean" or "sum"; the old
    `mean` flag still selects mean (True) or sum (False) when sync is None.

    hot_rows > 0 (sum rule only): the hub rows of each table -- the hot_rows
    rows with the highest expected touches per sample of `model`
    (smore_hot_row_ids) -- are also exchanged synchronously by hot(), which
    the caller runs after every training launch inside a step:

        D' = T_h - S_h;  R' = all_reduce(D');  T_h += R' - D';  S_h += R'

    This composes with the one-late full exchange (no update counted twice:
    the next begin() sees only the hub rows' changes since the last hot()).

    partition=True (LINE-2): rank r draws its sources from part r of the
    vertex ids (contiguous ranges of equal source mass,
    smore_set_source_partition), so each W row is updated by one rank only
    and only C is exchanged; end() then gathers W (each part broadcast from
    its owner).  The adaptive scales come from the global law.
    partition=True with model="census" (DeepWalk, Walklets, node2vec,
    metapath2vec, CTDNE after a row census): the walk partition -- this rank
    trains only the pairs whose center (W row) lies in its part of
    smore_walk_parts (smore_set_walk_owner), so EVERY rank runs EVERY walk of a
    step (the walks and draws are deterministic per walk index); only C is
    exchanged and W is gathered the same way."""

    def __init__(self, pn, mean=False, tables=(0, 1), group=None, hot_rows=0, model="line2", K=5, sync=None,
                 updates=None, c0=64.0, partition=False):
        # the passes, the training kernels and the collective must be ordered
        # on ONE stream.  The context runs on its own non-blocking stream when
        # handed the null stream (handle 0), which the legacy null stream does
        # not order against, so a dedicated torch stream is made current first.
        if torch.cuda.current_stream().cuda_stream == 0:
            torch.cuda.set_stream(torch.cuda.Stream())
        pn.set_stream(torch.cuda.current_stream().cuda_stream)
        if partition:
            if model not in ("line2", "census"):
                raise ValueError("partition: LINE-2 (sources) or a censused walk model (walk centers)")
            tables = (1,)
        T = [table_tensor(pn, w) for w in tables]
        if sync is None:
            sync = "mean" if mean else "sum"
        if sync not in ("sum", "mean", "adaptive"):
            raise ValueError("sync must be sum, mean or adaptive")
        row_scale = None
        if sync == "adaptive":
            if not updates:
                raise ValueError("the adaptive rule needs updates (samples per rank per exchange)")
            world = dist.get_world_size(group)
            row_scale = [torch.as_tensor(adaptive_scale(pn.row_rates(model, K, min(w, 1)), updates, world, c0),
                                         device=T[0].device) for w in tables]
        hot_idx = None
        if hot_rows > 0 and sync == "sum":
            n = min(int(hot_rows), pn.MAX_vid)
            hot_idx = [torch.as_tensor(pn.hot_row_ids(model, K, min(w, 1), n).astype("int64"), device=T[0].device)
                       for w in tables]
        super().__init__(T, mean=sync == "mean", group=group, passes=HipPasses(pn), hot_idx=hot_idx,
                         row_scale=row_scale)
        self.sync = sync
        self.bounds = None
        if partition:
            world, rank = dist.get_world_size(group), dist.get_rank(group)
            self.W = table_tensor(pn, 0)
            if model == "census":
                self.bounds = [int(b) for b in pn.walk_parts(world)]
                pn.set_walk_owner(self.bounds[rank], self.bounds[rank + 1])
            else:
                self.bounds = [int(b) for b in pn.source_parts(world)]
                pn.set_source_partition(world, rank)

    def gather_sources(self):
        """Every rank gets every part's W rows from the part's owner."""
        ranks = dist.get_process_group_ranks(self.group) if self.group is not None else None
        for p in range(len(self.bounds) - 1):
            lo, hi = self.bounds[p], self.bounds[p + 1]
            if hi > lo:
                dist.broadcast(self.W[lo:hi], src=ranks[p] if ranks else p, group=self.group)

    def end(self):
        super().end()
        if self.bounds is not None:
            self.gather_sources()
