"""Direct RCCL communicators for the data-parallel gradient all-reduce
(train_step.DataParallel, transport "rccl"): eager, between graph segments,
or captured inside the training step's HIP graph.

No collective of torch's ProcessGroupNCCL is ever issued by this package.
That process group keeps a watchdog thread that polls the completion event
of every collective it issued (hipEventQuery from another thread).  When the
stream that event was last recorded on is being captured at the time of the
poll -- a graph capture on a pooled torch stream that aliases the process
group's own stream, or a capture started before the watchdog reaped an
earlier collective -- the query fails with hipErrorCapturedEvent and the
watchdog aborts the process (round 5).  So:

  * the RCCL unique id travels through the process group's rendezvous STORE
    (a TCP key/value set/get, no device work), not through a broadcast;
  * every GPU collective of the steps goes through ncclAllReduce on the
    caller's stream, on a communicator of this module -- nothing polls it,
    and a graph replay re-issues the same RCCL launch;
  * the process group only carries host control (barriers, timings), and
    bench.py / the tests make it a gloo group.

The library is the librccl.so that torch itself links (torch/lib), so one
RCCL runs in the process; the RCCL API is plain C: ncclGetUniqueId,
ncclCommInitRank, ncclAllReduce, ncclCommDestroy.  One communicator per
process group (comm_for), made at its first use -- every rank reaches it at
the same collective point -- and released by release()."""
import ctypes
import os

import torch
import torch.distributed as dist

NCCL_FLOAT32 = 7   # ncclDataType_t ncclFloat32
NCCL_SUM = 0       # ncclRedOp_t ncclSum
UID_BYTES = 128    # NCCL_UNIQUE_ID_BYTES

_lib = None


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * UID_BYTES)]


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


def pack_uid(uid):
    """The id's 128 raw bytes.  (Not `bytes(uid.internal)`: ctypes cuts a
    c_char array at its first NUL, and RCCL's id -- a magic followed by a
    sockaddr -- holds zero bytes.)"""
    return ctypes.string_at(ctypes.addressof(uid), UID_BYTES)


def unpack_uid(raw):
    raw = bytes(raw)
    if len(raw) != UID_BYTES:
        raise ValueError("RCCL unique id: %d bytes, expected %d" % (len(raw), UID_BYTES))
    uid = _UniqueId()
    ctypes.memmove(ctypes.addressof(uid), raw, UID_BYTES)
    return uid


def _group_name(group):
    return "default" if group is None else str(getattr(group, "group_name", id(group)))


_seq = {}     # group name -> ids exchanged so far (the same sequence on every rank)


def exchange_uid(make_uid, group=None, store=None):
    """Rank 0's id bytes on every rank of `group`, through the rendezvous
    store: rank 0 sets key sgg_rccl_uid/<group>/<n>, the others block in
    get() until it is there.  make_uid() -> 128 bytes (called on rank 0
    only).  The n-th exchange of a group uses key n on every rank."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if world == 1:
        return make_uid()
    name = _group_name(group)
    n = _seq[name] = _seq.get(name, 0) + 1
    store = store if store is not None else dist.distributed_c10d._get_default_store()
    key = "sgg_rccl_uid/%s/%d" % (name, n)
    if rank == 0:
        raw = make_uid()
        store.set(key, raw)
        return raw
    return bytes(store.get(key))


def _new_uid():
    uid = _UniqueId()
    _check(_rccl().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    return pack_uid(uid)


class RcclComm:
    """One RCCL communicator over the ranks of `group` (an initialised
    torch.distributed process group of any backend: only its store and its
    rank numbering are used), on the current device."""

    def __init__(self, group=None):
        lib = _rccl()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        uid = unpack_uid(exchange_uid(_new_uid, group))
        comm = ctypes.c_void_p()
        _check(lib.ncclCommInitRank(ctypes.byref(comm), self.world, uid, self.rank), "ncclCommInitRank")
        self.comm = comm
        self.device = torch.cuda.current_device()

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
            torch.cuda.synchronize(self.device)
            _rccl().ncclCommDestroy(self.comm)
            self.comm = None


_comms = {}   # group name -> RcclComm


def comm_for(group=None):
    """The process's communicator over `group`, made at the first call (a
    collective point: every rank of the group must call it)."""
    name = _group_name(group)
    c = _comms.get(name)
    if c is None or c.comm is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("sgan.rccl: the communicator must exist before a graph capture "
                               "(DataParallel.prepare())")
        c = _comms[name] = RcclComm(group)
    return c


def release(group=None):
    """Destroy the communicator over `group` (every one when group is None);
    a collective point like comm_for.  Graphs that captured its all-reduce
    must be gone before."""
    names = list(_comms) if group is None else [_group_name(group)]
    for n in names:
        c = _comms.pop(n, None)
        if c is not None:
            c.destroy()
