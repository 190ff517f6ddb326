"""Pool forward on one training shape, for rocprofv3 counter passes.
usage: python tools/pool_probe.py [bn] [S] [reps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_kernels import run  # noqa: E402

bn = int(sys.argv[1]) if len(sys.argv) > 1 else 8
S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
run(S, 20, 32 if bn == 8 else 48, bn, gpws=(0,), reps=reps)
