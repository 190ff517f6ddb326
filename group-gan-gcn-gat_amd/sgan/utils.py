"""sgan.utils (reference sgan/utils.py)."""
import inspect
import os
import subprocess
import time
from contextlib import contextmanager

import numpy as np
import torch


def int_tuple(s):
    return tuple(int(i) for i in s.split(","))


def find_nan(variable, var_name):
    if np.isnan(variable.data.cpu().numpy()).any():
        exit("%s has nan" % var_name)


def bool_flag(s):
    if s == "1":
        return True
    if s == "0":
        return False
    raise ValueError('Invalid value "%s" for bool flag (should be 0 or 1)' % s)


def lineno():
    return str(inspect.currentframe().f_back.f_lineno)


def get_total_norm(parameters, norm_type=2):
    """utils.py:33-45, including its quirk: the running total is re-rooted
    after every parameter (so this is not the true global norm)."""
    if norm_type == float("inf"):
        return max(p.grad.data.abs().max() for p in parameters)
    total = 0
    for p in parameters:
        if p.grad is None:
            continue
        total += p.grad.data.norm(norm_type) ** norm_type
        total = total ** (1.0 / norm_type)
    return total


@contextmanager
def timeit(msg, should_time=True):
    if should_time:
        torch.cuda.synchronize()
        t0 = time.time()
    yield
    if should_time:
        torch.cuda.synchronize()
        print("%s: %.2f ms" % (msg, (time.time() - t0) * 1000.0))


def get_gpu_memory():
    """Used device memory in MiB (the reference shells out to nvidia-smi)."""
    torch.cuda.synchronize()
    try:
        out = subprocess.run(["rocm-smi", "--showmeminfo", "vram", "--json"], capture_output=True, text=True).stdout
        import json
        d = json.loads(out)
        card = sorted(d)[0]
        return int(int(d[card].get("VRAM Total Used Memory (B)", 0)) / 2 ** 20)
    except Exception:
        return int(torch.cuda.memory_allocated() / 2 ** 20)


def _data_root():
    env = os.environ.get("SGAN_DATASETS")
    if env:
        return env
    here = os.path.dirname(os.path.abspath(__file__))
    cands = [os.path.join(os.path.dirname(here), "datasets_group"),
             os.path.join(os.path.dirname(os.path.dirname(here)), "tests", "golden", "datasets_group")]
    for c in cands:
        if os.path.isdir(c):
            return c
    return cands[0]


def get_dset_path(dset_name, dset_type):
    """utils.py:75-80: <root>/datasets_group/<name>/<type>; the root is
    $SGAN_DATASETS, else a datasets_group/ next to the package (as in the
    reference), else the test splits shipped under tests/golden/."""
    return os.path.join(_data_root(), dset_name, dset_type)


def relative_to_abs(rel_traj, start_pos):
    """utils.py:83-96: cumulative sum of displacements from start_pos."""
    return (torch.cumsum(rel_traj.permute(1, 0, 2), dim=1) + start_pos.unsqueeze(1)).permute(1, 0, 2)
