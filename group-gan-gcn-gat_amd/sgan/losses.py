"""sgan.losses (reference sgan/losses.py): same functions, same host RNG use.

These are elementwise / reduction one-liners; they run as torch ops on
whatever device their inputs live on (the GPU in training).
"""
import random

import torch


def bce_loss(input, target):
    """losses.py:5-21: numerically stable BCE-with-logits, mean over the batch."""
    neg_abs = -input.abs()
    return (input.clamp(min=0) - input * target + (1 + neg_abs.exp()).log()).mean()


def gan_g_loss(scores_fake):
    """losses.py:24-33: one random.uniform(0.7, 1.2) label-smoothing draw."""
    return bce_loss(scores_fake, torch.ones_like(scores_fake) * random.uniform(0.7, 1.2))


def gan_d_loss(scores_real, scores_fake):
    """losses.py:36-49: two draws (real, then fake)."""
    y_real = torch.ones_like(scores_real) * random.uniform(0.7, 1.2)
    y_fake = torch.zeros_like(scores_fake) * random.uniform(0, 0.3)
    return bce_loss(scores_real, y_real) + bce_loss(scores_fake, y_fake)


def l2_loss(pred_traj, pred_traj_gt, loss_mask, random=0, mode="average"):
    """losses.py:52-71."""
    loss = loss_mask.unsqueeze(dim=2) * (pred_traj_gt.permute(1, 0, 2) - pred_traj.permute(1, 0, 2)) ** 2
    if mode == "sum":
        return torch.sum(loss)
    if mode == "average":
        return torch.sum(loss) / torch.numel(loss_mask.data)
    if mode == "raw":
        return loss.sum(dim=2).sum(dim=1)


def displacement_error(pred_traj, pred_traj_gt, consider_ped=None, mode="sum"):
    """losses.py:74-95."""
    d = torch.sqrt(((pred_traj_gt.permute(1, 0, 2) - pred_traj.permute(1, 0, 2)) ** 2).sum(dim=2)).sum(dim=1)
    if consider_ped is not None:
        d = d * consider_ped
    if mode == "sum":
        return torch.sum(d)
    if mode == "raw":
        return d


def final_displacement_error(pred_pos, pred_pos_gt, consider_ped=None, mode="sum"):
    """losses.py:98-119."""
    d = torch.sqrt(((pred_pos_gt - pred_pos) ** 2).sum(dim=1))
    if consider_ped is not None:
        d = d * consider_ped
    if mode == "raw":
        return d
    return torch.sum(d)
