"""Our TrajectoryDataset / seq_collate reproduce the reference's batches
bit-for-bit (fixture: first 16 zara1 test scenes as the reference built them)."""
import os

import numpy as np
import torch

from conftest import GOLDEN


def test_zara1_first_scenes_match_reference():
    from sgan.data.trajectories_GCN import TrajectoryDataset, seq_collate
    f = np.load(os.path.join(GOLDEN, "gen_fwd_gat.npz"))
    dset = TrajectoryDataset(os.path.join(GOLDEN, "datasets_group", "zara1", "test"))
    assert len(dset) == 602
    b = seq_collate([dset[i] for i in range(16)])
    names = ["obs_traj", "pred_traj", "obs_traj_rel", "pred_traj_rel", "obs_vel", "pred_vel", "obs_traj_g",
             "pred_traj_g", "non_linear_ped", "loss_mask", "seq_start_end"]
    got = dict(zip(names, b))
    for k in ("obs_traj", "obs_traj_rel", "obs_traj_g", "seq_start_end", "pred_traj", "pred_traj_rel"):
        np.testing.assert_array_equal(got[k].numpy(), f["zara1/" + k], err_msg=k)
    assert got["seq_start_end"].dtype == torch.int64
    assert torch.equal(got["obs_vel"], got["obs_traj_rel"] * 2.5)


def test_split_sizes_match_reference_eval():
    import json
    from sgan.data.trajectories_GCN import TrajectoryDataset
    ev = json.load(open(os.path.join(GOLDEN, "evaluate.json")))
    for split in ("eth", "hotel", "zara1"):
        dset = TrajectoryDataset(os.path.join(GOLDEN, "datasets_group", split, "test"))
        assert len(dset) == ev["gat/" + split]["num_seq"], split
