"""Pool forward: chunk-count target (-> gpw) at the bench's scene counts."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_kernels as BK  # noqa: E402
from sgan.scene import SceneIndex  # noqa: E402

for S, hd, bn in ((128, 48, 48), (64, 48, 48), (64, 32, 8)):
    for target in (128, 256, 512, 1024):
        SceneIndex.POOL_TARGET_CHUNKS = target
        print("target", target, end=": ", flush=True)
        BK.run(S, 20, hd, bn, gpws=(0,), reps=20)
