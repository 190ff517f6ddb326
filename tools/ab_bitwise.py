"""Bitwise A/B of two library builds on the benched configuration: 7 eager
paired iterations (tests/test_gpu_a_benched_path.py _run_configs1), weights
and losses saved; run once per build (SGG_LIB=...), then `cmp A B`."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "group-gan-gcn-gat_amd"))
import torch  # noqa: E402

if sys.argv[1] == "run":
    import test_gpu_a_benched_path as T  # noqa: E402
    losses, w = T._run_configs1(False)
    torch.save({"losses": losses, "w": w}, sys.argv[2])
    print("saved", sys.argv[2], losses)
else:
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    bad = [k for k in a["w"] if not torch.equal(a["w"][k], b["w"][k])]
    print("losses equal:", a["losses"] == b["losses"], "| weights differing:", len(bad), bad[:8])
    sys.exit(1 if bad or a["losses"] != b["losses"] else 0)
