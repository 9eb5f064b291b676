"""Diagnostic: library work first, then torch's first CUDA use (one process)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tests.test_gpu_parity as t  # noqa: E402

for args in [(61, 8, 2_000_000), (62, 3, 5000)]:
    t.test_merge_runs_and_split(*args)
import torch  # noqa: E402

print("torch after library:", torch.cuda.is_available(), torch.zeros(4, device="cuda").sum().item())
