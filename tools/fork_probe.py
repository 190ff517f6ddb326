"""Do forked branches of a captured HIP graph overlap on MI355X?  The
best-of-20 decoder rollout (25,600 no-grad sequences, batch-MFMA kernel) and
a discriminator-encoder forward (H 48, 2,560 peds, T 20, four-wave kernel)
captured (a) serially on one stream, (b) forked onto two streams (one fork,
one join), (c) each alone; device time per replay from HIP events over 200
back-to-back replays."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
import torch  # noqa: E402

from sgan import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    enc = torch.nn.LSTM(16, 48).to(dev)
    enc_e = torch.nn.Linear(2, 16).to(dev)
    dec = torch.nn.LSTM(16, 32).to(dev)
    dec_e = torch.nn.Linear(2, 16).to(dev)
    hp = torch.nn.Linear(32, 2).to(dev)
    rel_e = torch.randn(20, 2560, 2, device=dev)
    rel_d = torch.randn(25600, 2, device=dev)
    h0 = torch.randn(25600, 32, device=dev)

    def a():
        with torch.no_grad():
            K.lstm_sequence(rel_e, enc, enc_e)

    def b():
        with torch.no_grad():
            K.lstm_sequence(rel_d, dec, dec_e, h0=h0, proj=hp, decoder=True, T=12)

    for _ in range(3):
        a(), b()
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    pool = torch.cuda.graph_pool_handle()
    graphs = {}
    for name in ("a", "b", "serial", "forked"):
        g = torch.cuda.CUDAGraph()
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s0):
            g.capture_begin(pool=pool)
            if name == "a":
                a()
            elif name == "b":
                b()
            elif name == "serial":
                a()
                b()
            else:
                s1.wait_stream(s0)
                a()
                with torch.cuda.stream(s1):
                    b()
                s0.wait_stream(s1)
            g.capture_end()
        torch.cuda.current_stream().wait_stream(s0)
        graphs[name] = g
    torch.cuda.synchronize()
    # two graphs of 10 re-issues each (a: 10 x encoder, b: 10 x rollout),
    # replayed one after the other on one stream vs on two streams at once
    # (separate hardware queues, no dependency between them)
    g10 = {}
    for name, fn in (("a10", a), ("b10", b)):
        g = torch.cuda.CUDAGraph()
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s0):
            g.capture_begin(pool=pool)
            for _ in range(10):
                fn()
            g.capture_end()
        torch.cuda.current_stream().wait_stream(s0)
        g10[name] = g
    torch.cuda.synchronize()
    for rnd in range(2):
        for mode in ("one-stream", "two-streams"):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s0.wait_stream(torch.cuda.current_stream())
            s1.wait_stream(torch.cuda.current_stream())
            for _ in range(20):
                with torch.cuda.stream(s0):
                    g10["a10"].replay()
                with torch.cuda.stream(s1 if mode == "two-streams" else s0):
                    g10["b10"].replay()
            torch.cuda.current_stream().wait_stream(s0)
            torch.cuda.current_stream().wait_stream(s1)
            e1.record()
            e1.synchronize()
            print("round %d %-11s %.1f us per (a + b) pair" % (rnd, mode, e0.elapsed_time(e1) / 200 * 1e3), flush=True)
    for rnd in range(2):
        for name, g in graphs.items():
            for _ in range(5):
                g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                g.replay()
            e1.record()
            e1.synchronize()
            print("round %d %-7s %.1f us per replay" % (rnd, name, e0.elapsed_time(e1) / 200 * 1e3), flush=True)


if __name__ == "__main__":
    main()
