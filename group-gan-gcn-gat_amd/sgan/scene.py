"""Scene / group structure of a batch, built once per batch and kept on device.

The reference walks `seq_start_end` with a `.item()` per scene in every
module (sgan/models.py:257-258, 508-509, 640-641, 840-841) -- one device->host
sync per scene per module.  Here a batch's scenes become an int32 CSR
(`scene_off`, S+1) on the device, plus host copies of S, B and the largest
scene, computed ONCE per batch (one host read when seq_start_end lives on
the GPU, none when it is a CPU tensor as the DataLoader yields it).  The group
structure (models.py:263-278) is derived on device by sgg_group_index when a
module first asks for it and cached with the index.
"""
import numpy as np
import torch

from . import _native as N


class SceneIndex:
    def __init__(self, host_off, device, labels=None):
        host_off = np.asarray(host_off, dtype=np.int64)
        assert host_off.ndim == 1 and host_off[0] == 0 and np.all(np.diff(host_off) >= 0)
        self.host_off = host_off
        self.S = int(len(host_off) - 1)
        self.B = int(host_off[-1])
        sizes = np.diff(host_off)
        self.max_n = int(sizes.max()) if self.S else 0
        self.device = device
        self.scene_off = torch.from_numpy(host_off.astype(np.int32)).to(device, non_blocking=True)
        self._labels = labels
        self._groups = None

    # -- construction ------------------------------------------------------
    @staticmethod
    def from_seq_start_end(sse, device):
        a = sse.detach().to("cpu", torch.int64).numpy()  # one host read per batch
        if a.shape[0] == 0:
            return SceneIndex(np.zeros(1, np.int64), device)
        if not (a[0, 0] == 0 and np.all(a[1:, 0] == a[:-1, 1])):
            raise ValueError("seq_start_end must be contiguous and start at 0 (as seq_collate builds it)")
        return SceneIndex(np.concatenate([[0], a[:, 1]]), device)

    def repeat(self, k):
        """k back-to-back copies of the batch (sample-major): scene s of copy r
        is scene r*S + s.  Used to batch the best-of-k samples.  Memoised, so
        a captured graph never re-uploads the index."""
        reps = self.__dict__.setdefault("_reps", {})
        if k not in reps:
            off = np.concatenate([[0]] + [self.host_off[1:] + r * self.B for r in range(k)])
            reps[k] = SceneIndex(off, self.device)
        return reps[k]

    def ped_scene_long(self):
        """Scene of every ped as an int64 device tensor (noise broadcast)."""
        if getattr(self, "_ped_scene", None) is None:
            sizes = np.diff(self.host_off)
            self._ped_scene = torch.from_numpy(np.repeat(np.arange(self.S, dtype=np.int64), sizes)).to(
                self.device, non_blocking=True)
        return self._ped_scene

    def ped_scene_i32(self):
        """Scene of every ped as an int32 device tensor."""
        if getattr(self, "_ped_scene32", None) is None:
            sizes = np.diff(self.host_off)
            self._ped_scene32 = torch.from_numpy(np.repeat(np.arange(self.S, dtype=np.int32), sizes)).to(
                self.device, non_blocking=True)
        return self._ped_scene32

    POOL_TARGET_CHUNKS = int(__import__("os").environ.get("SGG_POOL_TARGET_CHUNKS", "512"))
    # bottlenecks <= 16 (the generator's pooling): two pair groups per wave
    # already at 256 chunks -- the fp32 fragment kernel then runs its grid in
    # one round of three workgroups per CU (LDS-bound) instead of 1.2 rounds:
    # 21.2 -> 18.3 us for the generator step's 2 x 64-scene pair (round 5,
    # tools/gpu_pool_target.sh; bn 48 keeps 512, where 256 picks 4 groups and
    # loses 2x)
    POOL_TARGET_CHUNKS_SMALL = int(__import__("os").environ.get("SGG_POOL_TARGET_CHUNKS_SMALL", "256"))
    POOL_MAX_GPW = int(__import__("os").environ.get("SGG_POOL_MAX_GPW", "0"))

    def pool_plan(self, bn, target_chunks=None, bf16=False):
        """Device chunk table for sgg_pool_fwd (built on the host by
        sgg_pool_plan, cached per bottleneck width); bf16: the table of
        sgg_pool_fwd_bf16 (sgg_pool_plan_bf16: big chunks, one per CU)."""
        target_chunks = target_chunks or (self.POOL_TARGET_CHUNKS_SMALL if bn <= 16 else self.POOL_TARGET_CHUNKS)
        plans = self.__dict__.setdefault("_pool_plans", {})
        key = (bn, target_chunks, self.POOL_MAX_GPW, bool(bf16))
        if key not in plans:
            import ctypes
            lib = N.load()
            off = np.ascontiguousarray(self.host_off.astype(np.int32))
            cap = int(self.B) + self.S + 1
            tab = np.zeros((cap, 4), dtype=np.int32)
            mr, gpw = ctypes.c_int(0), ctypes.c_int(0)
            if bf16:
                ncu = torch.cuda.get_device_properties(self.device).multi_processor_count \
                    if torch.device(self.device).type == "cuda" else 256
                nc = lib.sgg_pool_plan_bf16(off.ctypes.data_as(ctypes.c_void_p), self.S, bn, int(ncu),
                                            tab.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(mr),
                                            ctypes.byref(gpw))
            else:
                nc = lib.sgg_pool_plan(off.ctypes.data_as(ctypes.c_void_p), self.S, bn, target_chunks,
                                       self.POOL_MAX_GPW, tab.ctypes.data_as(ctypes.c_void_p), cap,
                                       ctypes.byref(mr), ctypes.byref(gpw))
            if nc < 0:
                N.check(nc, "sgg_pool_plan")
            dev = torch.from_numpy(tab[:max(nc, 1)].copy()).to(self.device, non_blocking=True)
            plans[key] = (dev, int(nc), int(mr.value), int(gpw.value))
        return plans[key]

    # -- groups ---------------------------------------------------------------
    def groups(self, labels):
        """Group structure from last-observation labels (B,) float on device."""
        key = (labels.data_ptr(), labels._version)
        if self._groups is not None and self._groups[0] == key:
            return self._groups[1]
        # (the cache entry keeps `labels` alive, so its address cannot be
        # recycled into different labels while the entry exists)
        lib = N.load()
        B, S = self.B, self.S
        dev = self.device
        lab = labels.contiguous().view(-1).float()
        assert lab.numel() == B
        ped_gid = torch.empty(B, dtype=torch.int32, device=dev)
        ped_scene = torch.empty(B, dtype=torch.int32, device=dev)
        group_off = torch.empty(S + 1, dtype=torch.int32, device=dev)
        group_scene = torch.zeros(max(B, 1), dtype=torch.int32, device=dev)
        group_count = torch.ones(max(B, 1), dtype=torch.int32, device=dev)
        ws = torch.empty(int(lib.sgg_group_index_ws(S, B)), dtype=torch.uint8, device=dev)
        N.check(lib.sgg_group_index(N.ptr(lab), N.ptr(self.scene_off), S, B, self.max_n, N.ptr(ped_gid),
                                    N.ptr(ped_scene), N.ptr(group_off), N.ptr(group_scene), N.ptr(group_count),
                                    N.ptr(ws), N.stream_ptr()), "sgg_group_index")
        g = Groups(self, lab, ped_gid, ped_scene, group_off, group_scene, group_count)
        self._groups = (key, g, labels)
        return g


class Groups:
    """Device-side group structure of a SceneIndex (all int32 unless noted).

    G (total groups) stays on the device (`n_groups_dev`); group-level buffers
    are sized B (the upper bound) and rows >= G are kept at zero, so nothing
    here needs a host sync."""

    def __init__(self, scenes, labels, ped_gid, ped_scene, group_off, group_scene, group_count):
        self.scenes = scenes
        self.labels = labels
        self.ped_gid = ped_gid
        self.ped_scene = ped_scene
        self.group_off = group_off
        self.group_scene = group_scene
        self.group_count = group_count
        self.n_groups_dev = group_off[scenes.S:]          # 1-element view, device
        self.cap = max(scenes.B, 1)                       # group rows allocated
        # 1/|g(i)| per ped (the R^T un-pool of the normalised R, models.py:286)
        self.ped_inv_size = group_count.index_select(0, ped_gid.long()).float().reciprocal()


# ---------------------------------------------------------------------------
# fixed-capacity scene index: HIP-graph replays over real batches
# ---------------------------------------------------------------------------
def padded_sizes(sizes, S_cap, B_cap, np_cap):
    """Scene sizes of a batch padded to exactly S_cap scenes / B_cap peds: the
    real scenes first, then S_cap - S padding scenes sharing the B_cap - B
    padding peds evenly (>= 1 each, so no scene is empty).  None when the
    batch does not fit (too many scenes or peds, a scene over np_cap, or too
    few padding peds for the padding scenes)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    S, B = len(sizes), int(sizes.sum())
    ps, pp = S_cap - S, B_cap - B
    if ps < 0 or pp < 0 or (S and sizes.max() > np_cap) or (ps == 0) != (pp == 0) or pp < ps \
            or pp > ps * np_cap:
        return None
    pad = np.full(ps, pp // ps if ps else 0, dtype=np.int64)
    pad[:pp - int(pad.sum())] += 1
    return np.concatenate([sizes, pad])


class PaddedScenes(SceneIndex):
    """A SceneIndex of fixed capacity -- S_cap scenes, B_cap peds, scenes of
    at most np_cap peds -- whose device arrays keep their addresses while
    load() refreshes their contents for each batch, so a training iteration
    captured in a HIP graph on it replays for every real batch that fits
    (sgan.train_step.BucketedGraphTrainer; the reference's loader yields
    batches of varying scene / ped counts, scripts/train.py:279-297).

    A batch is padded with extra scenes of zero-trajectory, zero-mask peds
    (padded_sizes; their input rows are -1 for sgg_gather_batch).  Padding
    scenes interact with nothing (message passing never crosses a scene);
    the losses leave them out: the L2 term of a scene without a masked step
    is 0 (sgg_l2_loss_*), and the BCE means run over the first `nvalid`
    scores of each range (sgg_bce_*, sgg_head_bwd) -- the real peds, which
    come first.  Everything the kernels read per batch lives in ONE packed
    int32 device buffer (nvalid | scene_off | ped scene | gather rows | the
    repeats' scene_off | per pooling plan its chunk count and table; the
    pooling kernels walk the device count, sgg_pool_fwd nchunks_dev),
    refreshed by one host-to-device copy per batch from alternating pinned
    staging buffers."""

    MAX_PLANS = 6

    def __init__(self, S_cap, B_cap, device, np_cap=64, reps=(2,), pool_cap=None):
        self.S, self.B, self.max_n = int(S_cap), int(B_cap), int(np_cap)
        self.device = device
        self._labels = self._groups = None
        self.reps = tuple(reps)
        # every chunk holds >= 1 row: a plan over the largest repeat never needs more
        self.pool_cap = int(pool_cap or max(self.reps + (1,)) * (self.B + self.S))
        o = 4
        self._lay = {"nvalid": 0, "scene_off": o}
        o += self.S + 1
        self._lay["ped_scene"] = o
        o += self.B
        self._lay["rows"] = o
        o += self.B
        for r in self.reps:
            self._lay["rep%d" % r] = o
            o += r * self.S + 1
        self._plan_base = o = (o + 3) & ~3
        self._plans = []                       # [(rep, bn, gpw)] registered, region k at plan_base + 4 k pool_cap
        self._total = o + self.MAX_PLANS * (4 + 4 * self.pool_cap)
        self._used = self._plan_base
        self._dev = torch.zeros(self._total, dtype=torch.int32, device=device)
        self._gpu = torch.device(device).type == "cuda"   # (a host-only index packs the same layout: tests)
        self._stage = [torch.zeros(self._total, dtype=torch.int32) for _ in range(2)]
        if self._gpu:
            self._stage = [t.pin_memory() for t in self._stage]
        self._stage_ev = [None, None]
        # graph staging buffers (load(graph_stage=i) / head_copy(i)); pinned
        # here: no host allocation may happen while a graph is captured
        self._gstage = [torch.zeros(self._total, dtype=torch.int32) for _ in range(2)]
        if self._gpu:
            self._gstage = [t.pin_memory() for t in self._gstage]
        self._cur = 0
        self.nvalid = self._dev[0:1]
        self.scene_off = self._view("scene_off", self.S + 1)
        self._ped32 = self._view("ped_scene", self.B)
        self.rows = self._view("rows", self.B)
        self._children = {}
        self.host_off = np.arange(self.S + 1, dtype=np.int64) * 0
        self._host_rows = None
        self._host_off_real = None

    def _view(self, name, n):
        o = self._lay[name]
        return self._dev[o:o + n]

    # -- SceneIndex API ------------------------------------------------------
    def repeat(self, k):
        if k == 1:
            return self
        if k not in self.reps:
            raise NotImplementedError("PaddedScenes: repeat(%d) not reserved (reps=%s)" % (k, self.reps))
        if k not in self._children:
            self._children[k] = _PaddedRepeat(self, k)
        return self._children[k]

    def ped_scene_i32(self):
        return self._ped32

    def ped_scene_long(self):
        raise NotImplementedError("PaddedScenes: no int64 ped-scene map (the fused decoder path does not use it)")

    def _plan_region(self, k):
        """Offset of plan k: [chunk count, 0, 0, 0 | pool_cap x (scene, i0, i1, gpw)]."""
        return self._plan_base + (4 + 4 * self.pool_cap) * k

    def pool_plan(self, bn, target_chunks=None, rep=1, bf16=False):
        """(chunk table, grid basis, max rows, gpw, device chunk count): the
        table holds up to pool_cap chunks; the kernels walk the device count,
        the grid is sized by the chunk count of the batch that registered the
        plan (the capture's)."""
        for k, (r, b, gpw, grid) in enumerate(self._plans):
            if (r, b) == (rep, bn):
                o = self._plan_region(k)
                tab = self._dev[o + 4:o + 4 + 4 * self.pool_cap].view(self.pool_cap, 4)
                return tab, grid, SGG_POOL_MAX_ROWS, gpw, self._dev[o:o + 1]
        # first use (warm-up, before capture): the chunk shape of this batch
        # by the normal heuristic, then fixed for every later batch
        if len(self._plans) >= self.MAX_PLANS:
            raise RuntimeError("PaddedScenes: more than %d pooling plans" % self.MAX_PLANS)
        off = self._rep_off(self.host_off, rep)
        _, nc, _, gpw = _plan(off, rep * self.S, bn, target_chunks or self.POOL_TARGET_CHUNKS, self.POOL_MAX_GPW,
                              self.pool_cap)
        self._plans.append((rep, bn, gpw, max(nc, 1)))
        self._used = self._plan_region(len(self._plans))
        if self._host_off_real is not None:    # fill the new region now (synchronously: before any capture)
            self.load(self._host_off_real, self._host_rows)
            if self._gpu:
                torch.cuda.current_stream(self.device).synchronize()
        return self.pool_plan(bn, rep=rep)

    def groups(self, labels):
        """The device group index of SceneIndex.groups, rebuilt on every call:
        the labels buffer is rewritten by each replay's batch gather behind
        torch's back, so no cached index may outlive a step."""
        self._groups = None
        return SceneIndex.groups(self, labels)

    # -- per batch -----------------------------------------------------------
    def _rep_off(self, off, r):
        return np.concatenate([[0]] + [off[1:] + k * self.B for k in range(r)]).astype(np.int64)

    def fits(self, sizes):
        return padded_sizes(sizes, self.S, self.B, self.max_n) is not None

    def pack(self, host_off_real, rows_real, out):
        """Fill `out` (int32, numpy, >= the used length) for a batch: real scene
        offsets host_off_real (S + 1) and its peds' table rows rows_real (B)."""
        sizes = padded_sizes(np.diff(host_off_real), self.S, self.B, self.max_n)
        if sizes is None:
            raise ValueError("PaddedScenes: batch (S=%d, B=%d, max n=%d) does not fit (S_cap=%d, B_cap=%d, "
                             "np_cap=%d)" % (len(host_off_real) - 1, int(host_off_real[-1]),
                                             int(np.diff(host_off_real).max()), self.S, self.B, self.max_n))
        off = np.concatenate([[0], np.cumsum(sizes)])
        B_r = int(host_off_real[-1])
        L = self._lay
        out[:self._used] = 0
        out[0] = B_r
        out[L["scene_off"]:L["scene_off"] + self.S + 1] = off
        out[L["ped_scene"]:L["ped_scene"] + self.B] = np.repeat(np.arange(self.S), sizes)
        r0 = L["rows"]
        out[r0:r0 + B_r] = rows_real
        out[r0 + B_r:r0 + self.B] = -1
        for r in self.reps:
            o = L["rep%d" % r]
            out[o:o + r * self.S + 1] = self._rep_off(off, r)
        for k, (r, bn, gpw, _) in enumerate(self._plans):
            o = self._plan_region(k)
            tab, nc, _, g = _plan(self._rep_off(off, r), r * self.S, bn, 0, gpw, self.pool_cap)
            assert g == gpw, (g, gpw)
            out[o] = nc
            out[o + 4:o + 4 + 4 * nc] = tab[:nc].reshape(-1)
        return off

    def _set_host(self, off, host_off_real, rows_real):
        self.host_off = off
        self._host_off_real, self._host_rows = host_off_real, np.asarray(rows_real, dtype=np.int32)
        for ch in self._children.values():
            ch.host_off = self._rep_off(self.host_off, ch.k)

    def _graph_stage(self):
        return self._gstage

    def head_copy(self, i):
        """The device arrays from graph staging buffer i (load(graph_stage=i)):
        captured at the head of graph i.  The used length is fixed by then (every
        pooling plan registers in the warm-up before the capture)."""
        self._dev[:self._used].copy_(self._graph_stage()[i][:self._used], non_blocking=True)

    def load(self, host_off_real, rows_real, graph_stage=None):
        """Refresh the device arrays for a batch: one asynchronous host-to-
        device copy on the current stream (graph replays issued after it read
        the new contents).

        graph_stage=i: only pack the batch into graph staging buffer i; the
        copy to the device is the head_copy(i) node captured at the start of
        graph i (BucketedGraphTrainer), and the caller has waited for graph
        i's previous replay.  No copy is issued from the host: a per-batch
        hipMemcpyAsync from the host stalled the thread for ~7 ms (4105 minor
        page faults inside the call) once every ~100 iterations
        (tools/realdata_stall_probe.py)."""
        if graph_stage is not None:
            host_off_real = np.asarray(host_off_real, dtype=np.int64)
            st = self._graph_stage()[graph_stage].numpy()
            self._set_host(self.pack(host_off_real, np.asarray(rows_real, dtype=np.int32), st), host_off_real,
                           rows_real)
            return
        i = self._cur
        self._cur ^= 1
        if self._stage_ev[i] is not None:
            self._stage_ev[i].synchronize()      # that staging buffer's previous copy has been consumed
        host_off_real = np.asarray(host_off_real, dtype=np.int64)
        st = self._stage[i].numpy()
        self._set_host(self.pack(host_off_real, np.asarray(rows_real, dtype=np.int32), st), host_off_real, rows_real)
        self._dev[:self._used].copy_(self._stage[i][:self._used], non_blocking=self._gpu)
        if self._gpu:
            ev = torch.cuda.Event()
            ev.record()
            self._stage_ev[i] = ev


class _PaddedRepeat(SceneIndex):
    """repeat(k) of a PaddedScenes: k back-to-back copies (the D-step's
    [fake | real] batch), views into the parent's packed buffer."""

    def __init__(self, parent, k):
        self.parent, self.k = parent, k
        self.S, self.B, self.max_n = k * parent.S, k * parent.B, parent.max_n
        self.device = parent.device
        self._labels = self._groups = None
        self.nvalid = parent.nvalid
        self.scene_off = parent._view("rep%d" % k, self.S + 1)
        self.host_off = parent._rep_off(parent.host_off, k)

    def repeat(self, k):
        raise NotImplementedError("repeat of a repeated PaddedScenes")

    def ped_scene_i32(self):
        raise NotImplementedError("PaddedScenes.repeat: no ped-scene map")

    def ped_scene_long(self):
        raise NotImplementedError("PaddedScenes.repeat: no ped-scene map")

    def pool_plan(self, bn, target_chunks=None, bf16=False):
        # (the fixed-capacity plan serves both precisions: the bf16 kernel takes any chunk table)
        return self.parent.pool_plan(bn, target_chunks, rep=self.k)

    def groups(self, labels):
        raise NotImplementedError("PaddedScenes: the per-op group index is not captured")


SGG_POOL_MAX_ROWS = 64   # chunk height bound of sgg_pool_fwd (a padded plan's LDS is sized for it)


def _plan(off, S, bn, target, max_gpw, cap):
    """sgg_pool_plan on a host offset array -> (table (cap x 4) int32, nchunks, max_rows, gpw)."""
    import ctypes
    lib = N.load(require_gpu=False)
    off = np.ascontiguousarray(np.asarray(off).astype(np.int32))
    tab = np.zeros((max(cap, 1), 4), dtype=np.int32)
    mr, gpw = ctypes.c_int(0), ctypes.c_int(0)
    nc = lib.sgg_pool_plan(off.ctypes.data_as(ctypes.c_void_p), S, bn, target, max_gpw,
                           tab.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(mr), ctypes.byref(gpw))
    if nc < 0:
        N.check(nc, "sgg_pool_plan")
    return tab, int(nc), int(mr.value), int(gpw.value)
