"""Helpers to read the golden .npz fixtures (bf16 payloads are uint16 bit patterns)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def tensor(arr):
    """uint16 -> bf16 tensor, float32 -> fp32 tensor, ints -> int64."""
    if arr.dtype == np.uint16:
        return torch.from_numpy(arr.astype(np.int16)).view(torch.bfloat16)
    if arr.dtype == np.float32:
        return torch.from_numpy(arr.copy())
    return torch.from_numpy(arr.astype(np.int64))
