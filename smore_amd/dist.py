"""Multi-GPU replication (new in this build; the reference is shared-memory
Hogwild only, src/model/LINE.cpp:162).

One process per GPU.  Every rank holds the whole graph and both embedding
tables, runs its own disjoint range of global sample indices (Hogwild inside
the GPU), and every few steps the ranks exchange what they learned:

    delta_r = T_r - T_snap ;  all_reduce(delta, SUM) over RCCL (xGMI)
    T = T_snap + sum_r delta_r      (or the mean, --sync mean)
    T_snap = T

With sum, every sample's update lands on the shared table exactly once --
the multi-GPU analogue of the reference's single shared table.  The
all-reduce works in place on the context's own device tables (zero-copy
through __cuda_array_interface__), one collective per table.
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
    """Snapshot-delta exchange over a list of same-shaped tensors on every rank."""

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


class ReplicaSync(DeltaAllReduce):
    """DeltaAllReduce over a ProNet context's device tables (W and C)."""

    def __init__(self, pn, mean=False, tables=(0, 1), group=None):
        super().__init__([table_tensor(pn, w) for w in tables], mean=mean, group=group)
