"""A direct RCCL communicator for the gradient all-reduce captured inside the
training step's HIP graph (train_step.DataParallel, capture=True).

torch's ProcessGroupNCCL keeps a watchdog thread that polls the completion
event of every collective it issues.  A collective issued while a graph is
being captured records that event inside the capture, and the watchdog's
poll of it (hipEventQuery from another thread) fails with
hipErrorCapturedEvent and invalidates the capture -- depending on when the
watchdog wakes, so in some runs only.  The captured
all-reduce therefore goes straight to RCCL: ncclAllReduce on the capturing
stream of a communicator of its own, made once from a unique id that rank 0
broadcasts over the existing process group.  Nothing polls it, and a graph
replay re-issues the same RCCL launch.

The library is the librccl.so that torch itself links (torch/lib), so one
RCCL runs in the process; the RCCL API is plain C: ncclGetUniqueId,
ncclCommInitRank, ncclAllReduce, ncclCommDestroy."""
import ctypes
import os

import torch
import torch.distributed as dist

NCCL_FLOAT32 = 7   # ncclDataType_t ncclFloat32
NCCL_SUM = 0       # ncclRedOp_t ncclSum

_lib = None


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]   # NCCL_UNIQUE_ID_BYTES


def _rccl():
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        lib = ctypes.CDLL(path)
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
        lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]
        lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        lib.ncclGetErrorString.argtypes = [ctypes.c_int]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclCommDestroy"):
            getattr(lib, f).restype = ctypes.c_int
        _lib = lib
    return _lib


def _check(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed: %s (ncclResult %d)" % (what, _rccl().ncclGetErrorString(rc).decode(), rc))


class RcclComm:
    """One RCCL communicator over the ranks of `group` (the process group of
    an initialised nccl backend), on the current device."""

    def __init__(self, group=None):
        lib = _rccl()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        box = [bytes(uid.internal)]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(box, src=src, group=group)
        uid.internal = box[0]
        comm = ctypes.c_void_p()
        _check(lib.ncclCommInitRank(ctypes.byref(comm), self.world, uid, self.rank), "ncclCommInitRank")
        self.comm = comm

    def allreduce_sum_(self, t):
        """In-place SUM all-reduce of a contiguous fp32 device tensor on the
        current stream (capturable)."""
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm.allreduce_sum_: a contiguous fp32 device tensor")
        if self.comm is None:
            raise RuntimeError("RcclComm: communicator destroyed")
        _check(_rccl().ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), NCCL_FLOAT32, NCCL_SUM, self.comm,
                                     torch.cuda.current_stream().cuda_stream), "ncclAllReduce")

    def destroy(self):
        if self.comm is not None:
            _rccl().ncclCommDestroy(self.comm)
            self.comm = None
