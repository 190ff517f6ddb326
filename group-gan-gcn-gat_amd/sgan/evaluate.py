"""Best-of-k evaluation (reference scripts/evaluate_model.py:58-99), batched.

The reference runs the generator num_samples times per batch, each call
drawing torch.randn((S, 8)) from the host RNG, then per scene takes the min
over samples of the summed per-ped errors.  Here the num_samples draws are
made in the same order from the same host generator and the samples run as
ONE generator call over a k-times replicated batch (sample-major scene
order); the reductions stay on the device.  Same ADE/FDE stream, one launch
sequence per batch instead of num_samples.
"""
import numpy as np
import torch

from .losses import displacement_error, final_displacement_error
from .models import get_noise
from .scene import SceneIndex
from .utils import relative_to_abs


def draw_sample_noise(generator, sc, B, k):
    """k consecutive host draws of the noise one reference generator call
    would make (models.py:827-835), concatenated sample-major."""
    if not generator.noise_dim:
        return None
    rows = sc.S if generator.noise_mix_type == "global" else B
    return torch.cat([get_noise((rows,) + tuple(generator.noise_dim), generator.noise_type) for _ in range(k)], 0)


def sample_k(generator, batch, k, sc=None):
    """k generator samples of a batch in one call -> pred_rel (pred_len, k, B, 2)."""
    (obs_traj, _pg, obs_traj_rel, _pr, _ov, _pv, obs_traj_g, _pgg, _nl, _lm, sse) = batch
    dev = obs_traj.device
    B = obs_traj.size(1)
    sc = sc or SceneIndex.from_seq_start_end(sse, dev)
    z = draw_sample_noise(generator, sc, B, k)
    if generator.pool_every_timestep and k > 1:   # per-step pooling: replicate the whole batch
        sck = sc.repeat(k)
        rep = lambda t: t.repeat(1, k, 1)
        sse_k = torch.from_numpy(np.stack([sck.host_off[:-1], sck.host_off[1:]], 1))
        out = generator(rep(obs_traj), rep(obs_traj_rel), sse_k, rep(obs_traj_g), user_noise=z, scenes=sck)
    else:   # the noise-independent context once, k decoder rollouts
        ctx = generator.context(obs_traj, obs_traj_rel, sse, obs_traj_g, scenes=sc)
        out = generator.decode(ctx, obs_traj, obs_traj_rel, sse, user_noise=z, scenes=sc, copies=k)
    return out.view(out.size(0), k, B, 2), sc


@torch.no_grad()
def evaluate(args, loader, generator, num_samples, device="cuda"):
    """Drop-in for scripts/evaluate_model.py:72-99; returns (ade, fde)."""
    ade_tot = torch.zeros((), dtype=torch.float64, device=device)
    fde_tot = torch.zeros((), dtype=torch.float64, device=device)
    total_traj = 0
    for batch in loader:
        if len(batch) == 2:          # sgan.data.device.DeviceLoader: (11-tuple on the device, SceneIndex)
            batch, sc = batch
        else:
            sc = SceneIndex.from_seq_start_end(batch[-1], device)   # host seq_start_end: no sync
        batch = [t.to(device, non_blocking=True) for t in batch]
        obs_traj, pred_gt = batch[0], batch[1]
        B = pred_gt.size(1)
        total_traj += B
        pred_rel, sc = sample_k(generator, batch, num_samples, sc)
        k = num_samples
        pr = pred_rel.reshape(pred_rel.size(0), k * B, 2)
        start = obs_traj[-1].repeat(k, 1)
        pred = relative_to_abs(pr, start)                                     # (T, kB, 2)
        gt = pred_gt.repeat(1, k, 1)
        ade = displacement_error(pred, gt, mode="raw").view(k, B)
        fde = final_displacement_error(pred[-1], gt[-1], mode="raw").view(k, B)
        seg = sc.ped_scene_long()
        ade_s = torch.zeros(k, sc.S, device=device).index_add_(1, seg, ade)
        fde_s = torch.zeros(k, sc.S, device=device).index_add_(1, seg, fde)
        ade_tot += ade_s.min(0)[0].double().sum()
        fde_tot += fde_s.min(0)[0].double().sum()
    return float(ade_tot) / (total_traj * args.pred_len), float(fde_tot) / total_traj


class _Args:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def evaluate_split(generator, path, num_samples=20, batch_size=64, obs_len=8, pred_len=12, device="cuda",
                   device_data=False):
    """Evaluate on one split directory with the reference's loader settings
    (shuffle=True, host RNG); device_data=True assembles the batches in HBM
    (sgan.data.device) in the same order."""
    a = _Args(obs_len=obs_len, pred_len=pred_len, skip=1, delim="tab", batch_size=batch_size, loader_num_workers=0)
    if device_data:
        from .data.device import device_data_loader
        _, loader = device_data_loader(a, path, device)
    else:
        from .data.loader import data_loader
        _, loader = data_loader(a, path)
    return evaluate(a, loader, generator, num_samples, device)
