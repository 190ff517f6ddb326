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

    POOL_TARGET_CHUNKS = 512
    POOL_MAX_GPW = int(__import__("os").environ.get("SGG_POOL_MAX_GPW", "0"))

    def pool_plan(self, bn, target_chunks=None):
        """Device chunk table for sgg_pool_fwd (built on the host by
        sgg_pool_plan, cached per bottleneck width)."""
        target_chunks = target_chunks or self.POOL_TARGET_CHUNKS
        plans = self.__dict__.setdefault("_pool_plans", {})
        key = (bn, target_chunks, self.POOL_MAX_GPW)
        if key not in plans:
            import ctypes
            lib = N.load()
            off = np.ascontiguousarray(self.host_off.astype(np.int32))
            cap = int(self.B) + self.S + 1
            tab = np.zeros((cap, 4), dtype=np.int32)
            mr, gpw = ctypes.c_int(0), ctypes.c_int(0)
            nc = lib.sgg_pool_plan(off.ctypes.data_as(ctypes.c_void_p), self.S, bn, target_chunks, self.POOL_MAX_GPW,
                                   tab.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(mr), ctypes.byref(gpw))
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
