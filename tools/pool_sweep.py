"""Pool-forward sweep: gpw and batch size for the discriminator pooling (bn 48)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_kernels import run  # noqa: E402

run(128, 20, 48, 48, gpws=(1, 2, 4))
run(64, 20, 48, 48, gpws=(1, 2, 4))
run(1024, 20, 48, 48, gpws=(1, 2, 4))
run(4096, 20, 48, 48, gpws=(2, 4))
run(64, 20, 32, 8, gpws=(1, 2))
run(4096, 20, 32, 8, gpws=(1, 2))
