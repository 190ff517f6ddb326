"""The bench's roofline launch alone (D pooling, 128 x 20-ped scenes, bn 48), for PMC passes."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_kernels import run  # noqa: E402

run(128, 20, 48, 48, gpws=(2,), reps=5)
