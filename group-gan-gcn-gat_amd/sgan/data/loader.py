"""sgan.data.loader (reference sgan/data/loader.py:9-29)."""
from torch.utils.data import DataLoader

from sgan.data.trajectories_GCN import TrajectoryDataset, seq_collate


def data_loader(args, path, shuffle=True):
    """(dataset, DataLoader) with shuffling from the host torch RNG, exactly
    as the reference (its RNG consumption defines the ADE/FDE sample stream)."""
    dset = TrajectoryDataset(path, obs_len=args.obs_len, pred_len=args.pred_len, skip=args.skip, delim=args.delim)
    loader = DataLoader(dset, batch_size=args.batch_size, shuffle=shuffle, num_workers=args.loader_num_workers,
                        collate_fn=seq_collate)
    return dset, loader
