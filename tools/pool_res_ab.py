"""Pool forward A/B on the training shapes: tiled (default), fragment-native
tiles (SGG_POOL_V=1), resident (SGG_POOL_RESIDENT=1)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_kernels import run  # noqa: E402

for name, env in (("tiled", {}), ("v", {"SGG_POOL_V": "1"}), ("resident", {"SGG_POOL_RESIDENT": "1"})):
    for k in ("SGG_POOL_V", "SGG_POOL_RESIDENT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    print(name, flush=True)
    run(64, 20, 32, 8, gpws=(0,))
    run(64, 20, 48, 48, gpws=(0,))
    run(128, 20, 48, 48, gpws=(0,))
    run(4096, 20, 48, 48, gpws=(0,))
