"""Which launches of one training iteration are not this library's kernels
(ATen glue: cat / fill / elementwise / reduce / copies) and where they come
from: torch.profiler over eager iterations of the bench's configs[1] step,
each non-sgg device kernel with the Python frames of the op that launched it.
usage: python tools/aten_glue.py"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "group-gan-gcn-gat_amd")]
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    trainer, batch, sc, batch_g, sc_g, kw = bench.setup(64, 20, 0, 1, dev, "gat")
    # the graph-mode step (device-resident RNG inputs, as GraphedTrainer replays it), run eagerly
    from sgan.train_step import GraphedTrainer
    gt = GraphedTrainer(trainer, batch, sc, warmup=2, batch_g=batch_g, sc_g=sc_g, **kw)
    gt._load(*trainer.draw_inputs(*gt.span))
    step = lambda: trainer.step(batch, sc, batch_g, sc_g, inputs=gt.inp, **gt.kw)   # noqa: E731
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 experimental_config=torch._C._profiler._ExperimentalConfig(verbose=True)) as prof:
        step()
        torch.cuda.synchronize()
    ev = prof.events()
    count = collections.Counter()
    where = collections.defaultdict(collections.Counter)
    for e in ev:
        if e.device_type != torch.autograd.DeviceType.CPU or e.name.startswith("sgg"):
            continue
        kids = [k for k in e.kernels] if hasattr(e, "kernels") else []
        if not kids:
            continue
        stack = [s for s in (e.stack or []) if "sgan" in s or "bench" in s or "train_step" in s][:5]
        for k in kids:
            if "sgg::" in k.name:
                continue
            key = (e.name, k.name[:70])
            count[key] += 1
            where[key][" <- ".join(stack)] += 1
    if not any(k for w in where.values() for k in w):
        print("(no python frames recorded)")
    for key, n in count.most_common():
        print("%3d  %-28s %s" % (n, key[0], key[1]))
        for st, m in where[key].most_common(4):
            print("        %2d  %s" % (m, st))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def callers():
    """Python call sites (file:line) of the torch calls that can launch glue
    kernels, over one graph-mode step run eagerly (sys.setprofile c_call)."""
    dev = torch.device("cuda", 0)
    trainer, batch, sc, batch_g, sc_g, kw = bench.setup(64, 20, 0, 1, dev, "gat")
    from sgan.train_step import GraphedTrainer
    gt = GraphedTrainer(trainer, batch, sc, warmup=2, batch_g=batch_g, sc_g=sc_g, **kw)
    gt._load(*trainer.draw_inputs(*gt.span))
    print("inputs:", type(gt.inp).__name__, [None if t is None else tuple(t.shape)
                                              for t in (gt.inp.z_d, gt.inp.z_g, gt.inp.y)])
    watch = {"full", "zeros", "ones", "cat", "stack", "to", "copy_", "sum", "add", "repeat", "contiguous", "clone",
             "tensor", "as_tensor", "zeros_like", "ones_like", "full_like", "index_add_", "where", "exp", "mul",
             "__mul__", "__add__", "__sub__", "__rmul__", "min", "fill_", "zero_", "reshape", "expand", "float"}
    seen = collections.Counter()

    def prof(frame, event, arg):
        if event == "c_call" and getattr(arg, "__name__", "") in watch:
            f = frame
            if "sgan" in f.f_code.co_filename or "train_step" in f.f_code.co_filename:
                seen["%s  %s:%d" % (arg.__name__, os.path.relpath(f.f_code.co_filename, ROOT), f.f_lineno)] += 1
    sys.setprofile(prof)
    trainer.step(batch, sc, batch_g, sc_g, inputs=gt.inp, **gt.kw)
    sys.setprofile(None)
    torch.cuda.synchronize()
    for k, n in sorted(seen.items(), key=lambda kv: kv[0].split()[1]):
        print("%3d  %s" % (n, k))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "callers":
    callers()
