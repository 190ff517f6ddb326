"""Synthetic scenes for benchmarks and tests (SURVEY.md §8d recipe): start
U[0,15)^2 m, per-ped velocity N(0, 0.3^2) m/step plus N(0, 0.05^2) jitter,
group labels uniform in {0..4} (0 = ungrouped), constant over time."""
import numpy as np
import torch


def synthetic_batch(sizes, seed=0, n_labels=5, obs_len=8, pred_len=12, device="cpu"):
    """11-tuple batch (seq_collate layout) of len(sizes) scenes."""
    rng = np.random.default_rng(seed)
    T = obs_len + pred_len
    B = int(sum(sizes))
    start = rng.uniform(0, 15, size=(B, 2))
    vel = rng.normal(0, 0.3, size=(B, 2))
    steps = vel[None] + rng.normal(0, 0.05, size=(T, B, 2))
    steps[0] = 0.0
    pos = start[None] + np.cumsum(steps, axis=0)
    rel = np.zeros_like(pos)
    rel[1:] = pos[1:] - pos[:-1]
    lab = rng.integers(0, n_labels, size=(B,)).astype(np.float64)
    g = np.broadcast_to(lab[None, :, None], (T, B, 1))
    off = np.concatenate([[0], np.cumsum(sizes)])
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a)).float().to(device)
    sse = torch.from_numpy(np.stack([off[:-1], off[1:]], 1).astype(np.int64)).to(device)
    return (f(pos[:obs_len]), f(pos[obs_len:]), f(rel[:obs_len]), f(rel[obs_len:]), f(rel[:obs_len] * 2.5),
            f(rel[obs_len:] * 2.5), f(g[:obs_len]), f(g[obs_len:]), torch.zeros(B, device=device),
            torch.ones(B, T, device=device), sse)
