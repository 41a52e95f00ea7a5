"""Image sources for the token optimisation and the keypoint stages.

- ``CelebA`` — reference ``datasets/celeba.py:8-150`` (aligned PNGs or in-the-wild JPEGs,
  MAFL train/test split files, 5 landmarks normalised by the image size as (row, col); the
  wild split drops images whose face box covers < 30 % of the image);
- ``CustomDataset`` — reference ``datasets/custom_images.py:7-28`` semantics (sorted
  folder listing, RGB, resize to 512² bilinear, [0, 1] float CHW), with PIL instead
  of torchvision;
- ``SyntheticDataset`` — seeded ``torch.rand`` images (the benchmark workload).

The other readers (CUB, Taichi, Human3.6M, DeepFashion) are not built.
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


class CelebA(torch.utils.data.Dataset):
    """datasets/celeba.py:8-150.  Layout under ``dataset_loc``: ``Anno/list_landmarks_align_celeba.txt``
    (or ``list_landmarks_celeba.txt`` and ``list_bbox_celeba.txt`` for the wild images),
    ``MAFL/training.txt`` / ``MAFL/testing.txt``, ``Img/img_align_celeba_png/NNNNNN.png`` or
    ``Img/img_celeba/NNNNNN.jpg``."""

    def __init__(self, max_len=-1, split="train", align=True, dataset_loc="~", iou_threshold=0.3):
        self.dataset_loc = os.path.expanduser(dataset_loc)
        self.max_len, self.align, self.split = max_len, align, split
        anno = os.path.join(self.dataset_loc, "Anno")
        with open(os.path.join(anno, "list_landmarks_align_celeba.txt" if align else "list_landmarks_celeba.txt")) as f:
            self.landmarks = f.readlines()
        listing = {"test": "testing.txt", "train": "training.txt"}[split]
        with open(os.path.join(self.dataset_loc, "MAFL", listing)) as f:
            self.file_names = f.readlines()
        self.num_kps = 5
        if not align:   # keep images whose face box covers at least iou_threshold of the image
            with open(os.path.join(anno, "list_bbox_celeba.txt")) as f:
                boxes = f.readlines()[2:]
            keep = []
            for name in self.file_names:
                k = self._index(name)
                _, _, bw, bh = (int(v) for v in boxes[k].split()[1:5])
                w, h = self._size(k)
                if bw * bh >= h * w * iou_threshold:
                    keep.append(name)
            self.file_names = keep

    @staticmethod
    def _index(name):
        return int(name.split(".")[0]) - 1   # 1-based file number → 0-based row

    def _path(self, k):
        name = f"{k + 1:06d}" + (".png" if self.align else ".jpg")
        sub = "img_align_celeba_png" if self.align else "img_celeba"
        return os.path.join(self.dataset_loc, "Img", sub, name)

    def _size(self, k):
        from PIL import Image
        with Image.open(self._path(k)) as im:
            return im.size

    def __len__(self):
        return self.max_len if self.max_len != -1 else len(self.file_names)

    def __getitem__(self, index):
        from PIL import Image
        k = self._index(self.file_names[index])
        with Image.open(self._path(k)) as im:
            w, h = im.size
            img = im.convert("RGB").resize((512, 512), Image.BILINEAR)
        img = torch.from_numpy(np.asarray(img).transpose(2, 0, 1).copy()) / 255.0
        xy = torch.tensor([float(v) for v in self.landmarks[k + 2].split()[1:]]).reshape(5, 2)
        kpts = (xy / torch.tensor([w, h]))[:, [1, 0]]
        return {"img": img, "kpts": kpts}


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


def make_dataset(name, loc="~", max_len=-1, validation=False, image_size=512, split="train"):
    if name in ("celeba_aligned", "celeba_wild"):
        return CelebA(max_len=max_len, split=split, align=(name == "celeba_aligned"), dataset_loc=loc)
    if name == "custom":
        ds = CustomDataset(loc, image_size)
    elif name == "synthetic":
        ds = SyntheticDataset(n=max_len if max_len > 0 else 64, size=image_size)
    else:
        raise NotImplementedError(f"dataset '{name}': readers built here are celeba_aligned, celeba_wild, custom and "
                                  "synthetic (or pass dataset=...)")
    if max_len > 0 and name == "custom":
        ds = torch.utils.data.Subset(ds, range(min(max_len, len(ds))))
    return ds
