"""Worker of test_gpu_parity.test_graphed_trainer_two_ranks and
test_gpu_configs.test_two_rank_512_scene_shard_equals_single (launched by
torch.distributed.run, 2 ranks sharing one GPU over gloo): the segmented
HIP-graph replay (GraphedTrainer, all-reduces between graph segments) must
match the eager scene-sharded GanTrainer step for step.

SGG_DP_SCENES=N: N synthetic 20-ped scenes as the global batch (default: a
6-scene ragged batch).  SGG_DP_VS_SINGLE=1: also run the whole global batch
on ONE rank (no data parallelism) and require the 2-rank result to equal it
(losses 1e-4 rel; weights within Adam's sign-flip bound on noise-level
gradients, 2 lr per step)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def models():
    from sgan.models import TrajectoryDiscriminator, TrajectoryGenerator
    torch.manual_seed(0)
    g = TrajectoryGenerator(8, 12, embedding_dim=16, encoder_h_dim=32, decoder_h_dim=32, mlp_dim=64,
                            noise_dim=(8,), noise_mix_type="global", pooling_type="pool_net",
                            pool_every_timestep=False, bottleneck_dim=8, batch_norm=False,
                            n_units=[40, 16, 40], n_heads=1, dropout1=0.0, alpha=0.2)
    d = TrajectoryDiscriminator(8, 12, embedding_dim=16, h_dim=48, mlp_dim=64, batch_norm=False, d_type="global")
    return g.cuda(), d.cuda()


def weights(g, d):
    """G and D state under distinct prefixes (both have an `encoder.`)."""
    out = {"g." + k: v.detach().cpu().clone() for k, v in g.state_dict().items()}
    out.update({"d." + k: v.detach().cpu().clone() for k, v in d.state_dict().items()})
    return out


def main():
    from sgan.data.synthetic import synthetic_batch
    from sgan.scene import SceneIndex
    from sgan.train_step import DataParallel, GanTrainer, GraphedTrainer, shard_batch
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    n_sc = int(os.environ.get("SGG_DP_SCENES", "0"))
    sizes = [20] * n_sc if n_sc else [20, 7, 13, 20, 2, 9]
    res = []
    hist = []
    for graphed in (False, True):
        g, d = models()
        tr = GanTrainer(g, d, dp=DataParallel())
        batch = synthetic_batch(sizes, seed=3, device="cuda")
        sc = SceneIndex(np.concatenate([[0], np.cumsum(sizes)]), "cuda")
        s0, s1 = tr.dp.shard(sc.S)
        local, lsc = shard_batch(batch, sc, s0, s1)
        kw = dict(S_global=sc.S, B_global=sc.B, shard=(s0, s1))
        torch.manual_seed(9)
        random.seed(9)
        if graphed:
            gt = GraphedTrainer(tr, local, lsc, warmup=2, **kw)
            assert len(gt.segments) == 3, len(gt.segments)
            for _ in range(2):
                ld, lg = gt.step()
        else:
            for _ in range(4):
                ld, lg = tr.step(local, lsc, **kw)
                hist.append([float(v) for v in list(ld.values()) + list(lg.values())])
        torch.cuda.synchronize()
        res.append(({k: float(v) for k, v in list(ld.items()) + list(lg.items())}, weights(g, d)))
    (la, wa), (lb, wb) = res
    for k in la:
        assert abs(la[k] - lb[k]) <= 1e-5 * max(1.0, abs(la[k])), (k, la[k], lb[k])
    for k in wa:
        err = (wa[k] - wb[k]).abs().max().item()
        assert err <= 1e-5 + 1e-5 * wa[k].abs().max().item(), (k, err)
    if os.environ.get("SGG_DP_VS_SINGLE") == "1":
        # the same 4 iterations on the WHOLE global batch, one rank, no DP
        g, d = models()
        dp1 = DataParallel()
        dp1.on, dp1.world, dp1.rank = False, 1, 0
        tr = GanTrainer(g, d, dp=dp1)
        batch = synthetic_batch(sizes, seed=3, device="cuda")
        sc = SceneIndex(np.concatenate([[0], np.cumsum(sizes)]), "cuda")
        torch.manual_seed(9)
        random.seed(9)
        for it in range(4):
            ld, lg = tr.step(batch, sc)
            one = [float(v) for v in list(ld.values()) + list(lg.values())]
            for a, b in zip(hist[it], one):
                assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), ("loss vs single rank", it, a, b)
        torch.cuda.synchronize()
        ws = weights(g, d)
        for k in ws:
            lr = 1e-3 if k.startswith("d.") else 1e-4
            err = (wa[k] - ws[k]).abs().max().item()
            assert err <= 2 * lr * 4 + 1e-5 * ws[k].abs().max().item(), ("weights vs single rank", k, err)
    dist.barrier()
    dist.destroy_process_group()
    print("rank %d OK" % int(os.environ["RANK"]), flush=True)


if __name__ == "__main__":
    main()
