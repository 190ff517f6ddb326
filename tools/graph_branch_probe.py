"""Do independent branches of a captured HIP graph run concurrently?  Two
discriminator-encoder sequences (H 48, 1,280 peds, T 20, four-wave kernel)
captured (a) on one stream and (b) forked onto two streams; replay times."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
import torch  # noqa: E402

from sgan import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    lstm = torch.nn.LSTM(16, 48).to(dev)
    emb = torch.nn.Linear(2, 16).to(dev)
    rel = [torch.randn(20, 1280, 2, device=dev) for _ in range(2)]

    def one(i):
        with torch.no_grad():
            return K.lstm_sequence(rel[i], lstm, emb)[0]

    for _ in range(3):
        one(0), one(1)
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    pool = torch.cuda.graph_pool_handle()
    g_ser, g_par = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        g_ser.capture_begin(pool=pool)
        one(0)
        one(1)
        g_ser.capture_end()
    with torch.cuda.stream(s0):
        g_par.capture_begin(pool=pool)
        s1.wait_stream(s0)
        one(0)
        with torch.cuda.stream(s1):
            one(1)
        s0.wait_stream(s1)
        g_par.capture_end()
    torch.cuda.current_stream().wait_stream(s0)
    torch.cuda.synchronize()
    for name, g in (("serial", g_ser), ("forked", g_par), ("serial", g_ser), ("forked", g_par)):
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            g.replay()
        torch.cuda.synchronize()
        print("%s: %.1f us per replay (2 launches)" % (name, (time.perf_counter() - t0) / 200 * 1e6), flush=True)


if __name__ == "__main__":
    main()
