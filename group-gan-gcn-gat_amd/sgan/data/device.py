"""Device-resident data path.

The reference rebuilds every batch on the host: DataLoader workers slice the
split's per-ped arrays, `seq_collate` (trajectories_GCN.py:15-42) permutes
and concatenates them, and the training loop copies the 11-tuple to the GPU
(scripts/train.py:396).  Here a split's peds are uploaded ONCE as a table in
HBM (one record of 6T + 1 floats per ped, layout in include/sgg.h) and a
batch is one gather launch (sgg_gather_batch) writing the time-major
11-tuple straight into device memory; the host only picks the scenes.

Batch order is the reference's: torch's RandomSampler (which draws its seed
from the host torch RNG once per epoch) feeding a BatchSampler, exactly what
`DataLoader(shuffle=True, batch_size=b)` does, so evaluation and training
see the same batches in the same order (and the same host RNG stream) as
through sgan.data.loader.data_loader.
"""
import numpy as np
import torch
from torch.utils.data import BatchSampler, RandomSampler, SequentialSampler

from .. import _native as N
from ..scene import SceneIndex
from .trajectories_GCN import TrajectoryDataset


class DeviceTrajectoryDataset:
    """A TrajectoryDataset's peds as one HBM table (built once per split)."""

    def __init__(self, dset, device="cuda"):
        self.dset = dset
        self.device = torch.device(device)
        self.obs_len, self.pred_len = dset.obs_len, dset.pred_len
        T = self.obs_len + self.pred_len
        P = dset.obs_traj.shape[0]
        absx = torch.cat([dset.obs_traj, dset.pred_traj], 2).permute(0, 2, 1)          # P x T x 2
        rel = torch.cat([dset.obs_traj_rel, dset.pred_traj_rel], 2).permute(0, 2, 1)    # P x T x 2
        grp = torch.cat([dset.obs_traj_g, dset.pred_traj_g], 2)[:, 0, :]                # P x T
        table = torch.cat([absx.reshape(P, 2 * T), rel.reshape(P, 2 * T), grp, dset.loss_mask,
                           dset.non_linear_ped.view(P, 1)], 1).float().contiguous()
        self.rec = table.shape[1]
        assert self.rec == 6 * T + 1
        self.table = table.to(self.device)
        self.scene_off = np.concatenate([[0], np.cumsum([e - s for s, e in dset.seq_start_end])]).astype(np.int64)

    def __len__(self):
        return len(self.dset)

    def layout(self, scenes):
        """(scene offsets (S + 1, int64), table rows of the batch's peds (B,
        int32)) of a batch of scene indices, on the host."""
        sizes = np.array([self.scene_off[s + 1] - self.scene_off[s] for s in scenes], dtype=np.int64)
        rows = np.concatenate([np.arange(self.scene_off[s], self.scene_off[s + 1]) for s in scenes]).astype(np.int32)
        return np.concatenate([[0], np.cumsum(sizes)]), rows

    def gather_into(self, rows_d, B, out):
        """sgg_gather_batch of B ped rows (device int32; < 0: padding) into out."""
        lib = N.load()
        N.check(lib.sgg_gather_batch(N.ptr(self.table), self.rec, N.ptr(rows_d), B, self.obs_len, self.pred_len,
                                     N.ptr(out), N.stream_ptr()), "sgg_gather_batch")

    def views(self, out, B, host_off):
        """The 11-tuple (seq_collate layout) as views of a gather buffer;
        seq_start_end on the host from host_off."""
        To, Tp = self.obs_len, self.pred_len
        T = To + Tp
        shapes = [(To, B, 2), (Tp, B, 2), (To, B, 2), (Tp, B, 2), (To, B, 2), (Tp, B, 2), (To, B, 1), (Tp, B, 1),
                  (B,), (B, T)]
        parts, o = [], 0
        for shp in shapes:
            n = int(np.prod(shp))
            parts.append(out[o:o + n].view(shp))
            o += n
        sse = torch.from_numpy(np.stack([host_off[:-1], host_off[1:]], 1).astype(np.int64))
        return tuple(parts) + (sse,)

    def batch(self, scenes):
        """11-tuple (seq_collate layout; every tensor on the device except
        seq_start_end, which stays on the host as the DataLoader yields it)
        and the batch's SceneIndex, for the given scene indices."""
        lib = N.load()
        off, rows = self.layout(scenes)
        B = int(rows.shape[0])
        rows_d = torch.from_numpy(rows).pin_memory().to(self.device, non_blocking=True)
        out = torch.empty(int(lib.sgg_gather_batch_floats(B, self.obs_len, self.pred_len)), device=self.device,
                          dtype=torch.float32)
        self.gather_into(rows_d, B, out)
        sc = SceneIndex(off, self.device)
        # keep the row list alive until the gather has consumed it
        sc._rows = rows_d
        return self.views(out, B, off), sc


class DeviceLoader:
    """Iterates (11-tuple, SceneIndex) batches of a DeviceTrajectoryDataset in
    the reference DataLoader's order (RandomSampler + BatchSampler)."""

    def __init__(self, ddset, batch_size=64, shuffle=True, drop_last=False):
        self.ddset, self.batch_size, self.shuffle, self.drop_last = ddset, batch_size, shuffle, drop_last
        self.dataset = ddset.dset

    def __len__(self):
        n = len(self.ddset)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        return (self.ddset.batch(scenes) for scenes in self.scene_batches())

    def scene_batches(self):
        """The batches as lists of scene indices (BucketedGraphTrainer gathers
        them itself into its fixed-capacity buffers)."""
        idx = range(len(self.ddset))
        sampler = RandomSampler(idx) if self.shuffle else SequentialSampler(idx)
        batches = iter(BatchSampler(sampler, self.batch_size, self.drop_last))
        # DataLoader's iterator draws its workers' base seed from the host
        # RNG when it is created (torch _BaseDataLoaderIter.__init__): so do we,
        # so the noise / shuffle stream matches the reference's loader
        torch.empty((), dtype=torch.int64).random_()
        return batches


def device_data_loader(args, path, device="cuda", shuffle=True):
    """(DeviceTrajectoryDataset, DeviceLoader) for a split directory, with the
    reference loader's windowing arguments (loader.py:9-29)."""
    dset = TrajectoryDataset(path, obs_len=args.obs_len, pred_len=args.pred_len, skip=args.skip, delim=args.delim)
    dd = DeviceTrajectoryDataset(dset, device)
    return dd, DeviceLoader(dd, batch_size=args.batch_size, shuffle=shuffle)
