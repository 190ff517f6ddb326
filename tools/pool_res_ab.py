"""Pool forward: tiled vs resident form (SGG_POOL_RESIDENT) on the training shapes."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_kernels import run  # noqa: E402

for res in ("0", "1"):
    os.environ["SGG_POOL_RESIDENT"] = res
    print("SGG_POOL_RESIDENT=" + res, flush=True)
    run(64, 20, 32, 8, gpws=(1, 2))
    run(64, 20, 48, 48, gpws=(1, 2))
    run(128, 20, 48, 48, gpws=(1, 2, 4))
