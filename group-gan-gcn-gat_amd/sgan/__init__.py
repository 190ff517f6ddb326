"""MI355X-native re-implementation of the group-aware Social-GAN hot path
(reference: peaceminusones/Group-GAN-GCN-GAT, package `sgan`).

Import layout mirrors the reference: sgan.models, sgan.losses, sgan.utils,
sgan.data.loader / sgan.data.trajectories_GCN.
"""
__version__ = "0.1.0"
