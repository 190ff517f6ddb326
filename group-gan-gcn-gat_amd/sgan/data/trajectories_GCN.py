"""Trajectory windows with group labels (reference sgan/data/trajectories_GCN.py).

Same windowing, same 11-tuple batches (the drop-in data contract), written
as host numpy preprocessing (one-off per split).  Input rows are
`frame ped x y group` separated by TABs (the reference splits on TAB whatever
`delim` says, trajectories_GCN.py:53).
"""
import logging
import math
import os

import numpy as np
import torch
from torch.utils.data import Dataset

logger = logging.getLogger(__name__)

_COLLATE_ORDER = ("obs_traj", "pred_traj", "obs_traj_rel", "pred_traj_rel", "obs_vel", "pred_vel",
                  "obs_traj_g", "pred_traj_g", "non_linear_ped", "loss_mask", "seq_start_end")


def seq_collate(data):
    """trajectories_GCN.py:15-42: concatenate scenes along the ped axis,
    time-major (T, B, d) tensors, seq_start_end (S, 2) int64."""
    cols = list(zip(*data))
    sizes = [len(x) for x in cols[0]]
    starts = np.concatenate([[0], np.cumsum(sizes)])
    sse = torch.LongTensor(np.stack([starts[:-1], starts[1:]], axis=1).tolist())
    tm = [torch.cat(c, dim=0).permute(2, 0, 1) for c in cols[:8]]   # (B, d, T) -> (T, B, d)
    non_linear_ped = torch.cat(cols[8])
    loss_mask = torch.cat(cols[9], dim=0)
    return tuple(tm + [non_linear_ped, loss_mask, sse])


def read_file(_path, delim="\t"):
    """trajectories_GCN.py:45-56 (always TAB-separated)."""
    rows = []
    with open(_path, "r") as f:
        for line in f:
            rows.append([float(v) for v in line.strip().split("\t")])
    return np.asarray(rows)


def poly_fit(traj, traj_len, threshold):
    """trajectories_GCN.py:59-74: 1.0 if a quadratic fit of the last traj_len
    points leaves residual >= threshold (non-linear), else 0.0."""
    t = np.linspace(0, traj_len - 1, traj_len)
    res_x = np.polyfit(t, traj[0, -traj_len:], 2, full=True)[1]
    res_y = np.polyfit(t, traj[1, -traj_len:], 2, full=True)[1]
    return 1.0 if res_x + res_y >= threshold else 0.0


class TrajectoryDataset(Dataset):
    """trajectories_GCN.py:77-204.  A scene = the peds present in all seq_len
    consecutive frames of a window starting at every `skip`-th frame; scenes
    with more than `min_ped` such peds are kept.  Files are read in sorted
    order (the reference's os.listdir order on its checkout)."""

    def __init__(self, data_dir, obs_len=8, pred_len=12, skip=1, threshold=0.002, min_ped=1, delim="\t",
                 files=None):
        super().__init__()
        self.data_dir = data_dir
        self.obs_len, self.pred_len, self.skip = obs_len, pred_len, skip
        self.seq_len = obs_len + pred_len
        self.delim = delim
        T = self.seq_len
        names = files if files is not None else sorted(os.listdir(data_dir))
        seqs, rels, grps, masks, nonlin, counts = [], [], [], [], [], []
        for name in names:
            data = read_file(os.path.join(data_dir, name), delim)
            frames = np.unique(data[:, 0]).tolist()
            frame_pos = {f: k for k, f in enumerate(frames)}
            by_frame = [data[data[:, 0] == f, :] for f in frames]
            n_windows = int(math.ceil((len(frames) - T + 1) / skip))
            for idx in range(0, n_windows * skip + 1, skip):
                window = by_frame[idx:idx + T]
                if not window:
                    continue
                cur = np.concatenate(window, axis=0)
                kept_seq, kept_rel, kept_g, kept_nl = [], [], [], []
                for ped in np.unique(cur[:, 1]):
                    ps = np.around(cur[cur[:, 1] == ped, :], decimals=4)
                    front = frame_pos[ps[0, 0]] - idx
                    end = frame_pos[ps[-1, 0]] - idx + 1
                    if end - front != T or ps.shape[0] != T:
                        continue
                    tr = ps[:, 2:].T                         # (3, T): x, y, group
                    assert tr.shape[0] == 3, "dataset has no labeling"
                    rel = np.zeros((2, T))
                    rel[:, 1:] = tr[:2, 1:] - tr[:2, :-1]
                    kept_seq.append(tr[:2])
                    kept_rel.append(rel)
                    kept_g.append(tr[2:])
                    kept_nl.append(poly_fit(tr, pred_len, threshold))
                n = len(kept_seq)
                if n > min_ped:
                    counts.append(n)
                    seqs.append(np.stack(kept_seq))
                    rels.append(np.stack(kept_rel))
                    grps.append(np.stack(kept_g))
                    masks.append(np.ones((n, T)))
                    nonlin += kept_nl
        self.num_seq = len(seqs)
        seq = np.concatenate(seqs, axis=0)
        rel = np.concatenate(rels, axis=0)
        grp = np.concatenate(grps, axis=0)
        f = lambda a: torch.from_numpy(a).type(torch.float)
        self.obs_traj = f(seq[:, :, :obs_len])
        self.pred_traj = f(seq[:, :, obs_len:])
        self.obs_traj_rel = f(rel[:, :, :obs_len])
        self.pred_traj_rel = f(rel[:, :, obs_len:])
        self.obs_traj_g = f(grp[:, :, :obs_len])
        self.pred_traj_g = f(grp[:, :, obs_len:])
        self.loss_mask = f(np.concatenate(masks, axis=0))
        self.non_linear_ped = f(np.asarray(nonlin))
        starts = np.concatenate([[0], np.cumsum(counts)]).tolist()
        self.seq_start_end = list(zip(starts[:-1], starts[1:]))

    def __len__(self):
        return self.num_seq

    def __getitem__(self, index):
        s, e = self.seq_start_end[index]
        return [
            self.obs_traj[s:e, :], self.pred_traj[s:e, :],
            self.obs_traj_rel[s:e, :], self.pred_traj_rel[s:e, :],
            self.obs_traj_rel[s:e, :] * 2.5, self.pred_traj_rel[s:e, :] * 2.5,   # velocity (/0.4 s)
            self.obs_traj_g[s:e, :], self.pred_traj_g[s:e, :],
            self.non_linear_ped[s:e], self.loss_mask[s:e, :],
        ]
