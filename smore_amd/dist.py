"""Multi-GPU replication (new in this build; the reference is shared-memory
Hogwild only, src/model/LINE.cpp:162).

One process per GPU.  Every rank holds the whole graph and both embedding
tables, runs its own disjoint range of global sample indices (Hogwild inside
the GPU), and the ranks exchange what they learned through the snapshot-delta
rule

    delta_r = T_r - T_snap ;  all_reduce(delta, SUM) over RCCL (xGMI)
    T = T_snap + sum_r delta_r      (or the mean, --sync mean)

With sum, every sample's update lands on every replica exactly once -- the
multi-GPU analogue of the reference's single shared table.

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
        self.pn.delta_end(T.data_ptr(), S.data_ptr(), D.data_ptr(), R.data_ptr(), scale, T.numel())

    def cycle(self, T, S, D, R, scale):
        self.pn.delta_cycle(T.data_ptr(), S.data_ptr(), D.data_ptr(), R.data_ptr(), scale, T.numel())


class OverlapSync:
    """One-exchange-late snapshot-delta exchange whose collective overlaps the
    next compute step (see the module docstring).

        begin():  [end() of the previous exchange, fused with this begin];
                  D = T - S; R = D; S = T; all_reduce(R) started asynchronously
        end():    wait for the collective; X = scale*R - D; T += X; S += X

    After end() every replica holds every rank's updates up to the matching
    begin(), plus its own since."""

    def __init__(self, tensors, mean=False, group=None, passes=None):
        self.T = list(tensors)
        self.S = [t.clone() for t in self.T]
        self.D = [torch.zeros_like(t) for t in self.T]
        self.R = [torch.zeros_like(t) for t in self.T]
        self.mean = mean
        self.group = group
        self.passes = passes or TorchPasses()
        self.works = None

    def begin(self):
        if self.works is not None:      # fold the previous exchange in and start this one: one pass
            for w in self.works:
                w.wait()
            scale = self._scale()
            for T, S, D, R in zip(self.T, self.S, self.D, self.R):
                self.passes.cycle(T, S, D, R, scale)
        else:
            for T, S, D, R in zip(self.T, self.S, self.D, self.R):
                self.passes.begin(T, S, D, R)
        self.works = [dist.all_reduce(R, op=dist.ReduceOp.SUM, group=self.group, async_op=True) for R in self.R]

    def _scale(self):
        return 1.0 / dist.get_world_size(self.group) if self.mean else 1.0

    def end(self):
        if self.works is None:
            return
        for w in self.works:
            w.wait()
        scale = self._scale()
        for T, S, D, R in zip(self.T, self.S, self.D, self.R):
            self.passes.end(T, S, D, R, scale)
        self.works = None

    def allreduce(self):
        """Synchronous use: begin() then end()."""
        self.begin()
        self.end()


class ReplicaSync(OverlapSync):
    """OverlapSync over a ProNet context's device tables (W and C), with the
    fused HIP passes; the context runs on torch's current stream so the
    passes, the training kernels and the collective are ordered on it."""

    def __init__(self, pn, mean=False, tables=(0, 1), group=None):
        # the passes, the training kernels and the collective must be ordered
        # on ONE stream.  The context runs on its own non-blocking stream when
        # handed the null stream (handle 0), which the legacy null stream does
        # not order against, so a dedicated torch stream is made current first.
        if torch.cuda.current_stream().cuda_stream == 0:
            torch.cuda.set_stream(torch.cuda.Stream())
        pn.set_stream(torch.cuda.current_stream().cuda_stream)
        super().__init__([table_tensor(pn, w) for w in tables], mean=mean, group=group, passes=HipPasses(pn))
