"""Image sources for the token-optimisation loop.

The reference's dataset readers (``datasets/*.py``: CelebA, CUB, Taichi, Human3.6M,
DeepFashion) are file I/O outside the hot path.  This module
provides the two sources the path and its benchmarks need:

- ``CustomDataset`` — reference ``datasets/custom_images.py:7-28`` semantics (sorted
  folder listing, RGB, resize to 512² bilinear, [0, 1] float CHW), with PIL instead
  of torchvision;
- ``SyntheticDataset`` — seeded ``torch.rand`` images (the benchmark workload).
"""
import os

import numpy as np
import torch


class CustomDataset(torch.utils.data.Dataset):
    def __init__(self, data_root, image_size=512):
        super().__init__()
        self.data_root = os.path.expanduser(data_root)
        self.image_files = sorted(f for f in os.listdir(self.data_root)
                                  if os.path.isfile(os.path.join(self.data_root, f)))
        self.image_size = image_size

    def __getitem__(self, idx):
        from PIL import Image
        img = Image.open(os.path.join(self.data_root, self.image_files[idx])).convert("RGB")
        img = img.resize((self.image_size, self.image_size), Image.BILINEAR)
        t = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1).contiguous()
        return {"img": t, "kpts": torch.zeros(15, 2), "visibility": torch.zeros(15)}

    def __len__(self):
        return len(self.image_files)


class SyntheticDataset(torch.utils.data.Dataset):
    """``n`` images ``torch.rand(3, size, size)`` from a fixed seed (per-index generator)."""

    def __init__(self, n=64, size=512, seed=0):
        self.n, self.size, self.seed = n, size, seed

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + int(idx))
        return {"img": torch.rand(3, self.size, self.size, generator=g), "kpts": torch.zeros(15, 2),
                "visibility": torch.zeros(15)}

    def __len__(self):
        return self.n


def make_dataset(name, loc="~", max_len=-1, validation=False, image_size=512):
    if name == "custom":
        ds = CustomDataset(loc, image_size)
    elif name == "synthetic":
        ds = SyntheticDataset(n=max_len if max_len > 0 else 64, size=image_size)
    else:
        raise NotImplementedError(f"dataset '{name}': the reference's file readers are outside the ported hot path; "
                                  "use dataset_name='custom' (an image folder) or 'synthetic', or pass dataset=...")
    if max_len > 0 and name == "custom":
        ds = torch.utils.data.Subset(ds, range(min(max_len, len(ds))))
    return ds
