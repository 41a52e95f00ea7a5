"""Image sources for the token optimisation and the keypoint stages.

- ``CelebA`` — reference ``datasets/celeba.py:8-150`` (aligned PNGs or in-the-wild JPEGs,
  MAFL train/test split files, 5 landmarks normalised by the image size as (row, col); the
  wild split drops images whose face box covers < 30 % of the image);
- ``CustomDataset`` — reference ``datasets/custom_images.py:7-28`` semantics (sorted
  folder listing, RGB, resize to 512² bilinear, [0, 1] float CHW), with PIL instead
  of torchvision;
- ``SyntheticDataset`` — seeded ``torch.rand`` images (the benchmark workload).

- ``CUBParts`` — reference ``datasets/cub_parts.py:242-440`` (``cub_001`` / ``cub_002`` /
  ``cub_003`` / ``cub_all``): CMR-style ``.mat`` annotations, padded (and, for training, jittered)
  square bounding-box crop, scale to 512, random mirror with the part permutation, 15 parts.

The other readers (``cub_aligned``'s ``cub.h5`` needs h5py, absent here; Taichi, Human3.6M,
DeepFashion) are not built.
"""
import math
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


# ------------------------------------------------------------------------------------------ CUB
CUB_PADDING_FRAC = 0.05   # cub_parts.py:21-22
CUB_JITTER_FRAC = 0.05
CUB_KP_PERM = np.array([1, 2, 3, 4, 5, 6, 11, 12, 13, 10, 7, 8, 9, 14, 15]) - 1   # left/right parts swap


def _quaternion_matrix(q):
    """cub_parts.py:23-48: 4×4 homogeneous rotation of quaternion (w, x, y, z)."""
    q = np.array(q, dtype=np.float64, copy=True)
    n = float(np.dot(q, q))
    if n < np.finfo(float).eps * 4.0:
        return np.identity(4)
    q *= math.sqrt(2.0 / n)
    q = np.outer(q, q)
    return np.array([[1.0 - q[2, 2] - q[3, 3], q[1, 2] - q[3, 0], q[1, 3] + q[2, 0], 0.0],
                     [q[1, 2] + q[3, 0], 1.0 - q[1, 1] - q[3, 3], q[2, 3] - q[1, 0], 0.0],
                     [q[1, 3] - q[2, 0], q[2, 3] + q[1, 0], 1.0 - q[1, 1] - q[2, 2], 0.0],
                     [0.0, 0.0, 0.0, 1.0]])


def _quaternion_from_rotation(M):
    """cub_parts.py:51-133 with isprecise=True (the only form the dataset calls): quaternion
    (w, x, y, z), w >= 0, of a 4×4 homogeneous rotation."""
    M = np.asarray(M, dtype=np.float64)[:4, :4]
    q = np.empty(4)
    t = np.trace(M)
    if t > M[3, 3]:
        q[0] = t
        q[3] = M[1, 0] - M[0, 1]
        q[2] = M[0, 2] - M[2, 0]
        q[1] = M[2, 1] - M[1, 2]
    else:
        i, j, k = 0, 1, 2
        if M[1, 1] > M[0, 0]:
            i, j, k = 1, 2, 0
        if M[2, 2] > M[i, i]:
            i, j, k = 2, 0, 1
        t = M[i, i] - (M[j, j] + M[k, k]) + M[3, 3]
        q[i] = t
        q[j] = M[i, j] + M[j, i]
        q[k] = M[k, i] + M[i, k]
        q[3] = M[k, j] - M[j, k]
        q = q[[3, 0, 1, 2]]
    q *= 0.5 / math.sqrt(t * M[3, 3])
    if q[0] < 0.0:
        q = -q
    return q


def _perturb_bbox(bbox, pf, jf, rng):
    """cub_parts.py:144-164: pad by pf and jitter by jf (uniform in ±jf) of the box size; the
    four uniform draws happen even when jf = 0, as the reference's do."""
    b = list(bbox)
    bw, bh = bbox[2] - bbox[0] + 1, bbox[3] - bbox[1] + 1
    b[0] -= pf * bw + (1 - 2 * rng.random()) * jf * bw
    b[1] -= pf * bh + (1 - 2 * rng.random()) * jf * bh
    b[2] += pf * bw + (1 - 2 * rng.random()) * jf * bw
    b[3] += pf * bh + (1 - 2 * rng.random()) * jf * bh
    return b


def _square_bbox(bbox):
    """cub_parts.py:167-184: grow the shorter side symmetrically to a square."""
    sq = [int(round(c)) for c in bbox]
    bw, bh = sq[2] - sq[0] + 1, sq[3] - sq[1] + 1
    maxdim = float(max(bw, bh))
    sq[0] -= int(round((maxdim - bw) / 2.0))
    sq[1] -= int(round((maxdim - bh) / 2.0))
    sq[2] = sq[0] + maxdim - 1
    sq[3] = sq[1] + maxdim - 1
    return sq


def _crop(img, bbox, bgval=0.0):
    """cub_parts.py:187-218: crop (float64 out, regions outside the image filled with bgval)."""
    bbox = [int(round(c)) for c in bbox]
    bw, bh = bbox[2] - bbox[0] + 1, bbox[3] - bbox[1] + 1
    h, w = img.shape[:2]
    nc = 1 if img.ndim < 3 else img.shape[2]
    out = np.ones((bh, bw, nc)) * bgval
    xs0, xs1 = max(0, bbox[0]), min(w, bbox[2] + 1)
    ys0, ys1 = max(0, bbox[1]), min(h, bbox[3] + 1)
    xt0, yt0 = xs0 - bbox[0], ys0 - bbox[1]
    src = img if img.ndim == 3 else img[:, :, None]
    out[yt0:yt0 + (ys1 - ys0), xt0:xt0 + (xs1 - xs0), :] = src[ys0:ys1, xs0:xs1, :]
    return out


def _resize_linear(img, new_h, new_w):
    """cv2.resize(..., INTER_LINEAR) on float input: half-pixel source coordinates
    (dst + 0.5)·(src/dst) − 0.5, taps clamped at the borders, no antialiasing."""
    h, w = img.shape[:2]

    def axis(n_out, n_in):
        f = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
        i0 = np.floor(f).astype(np.int64)
        t = f - i0
        t = np.where(i0 < 0, 0.0, t)
        i0 = np.clip(i0, 0, n_in - 1)
        t = np.where(i0 >= n_in - 1, 0.0, t)
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, t

    y0, y1, ty = axis(new_h, h)
    x0, x1, tx = axis(new_w, w)
    ty = ty[:, None, None]
    tx = tx[None, :, None]
    im = img if img.ndim == 3 else img[:, :, None]
    top = im[y0][:, x0] * (1 - tx) + im[y0][:, x1] * tx
    bot = im[y1][:, x0] * (1 - tx) + im[y1][:, x1] * tx
    out = top * (1 - ty) + bot * ty
    return out if img.ndim == 3 else out[:, :, 0]


def _resize_nearest(img, new_h, new_w):
    """cv2.resize(..., INTER_NEAREST): source index floor(dst · src/dst), clamped."""
    h, w = img.shape[:2]
    ys = np.minimum(np.floor(np.arange(new_h) * (h / new_h)).astype(np.int64), h - 1)
    xs = np.minimum(np.floor(np.arange(new_w) * (w / new_w)).astype(np.int64), w - 1)
    return img[ys][:, xs]


class CUBParts(torch.utils.data.Dataset):
    """datasets/cub_parts.py:242-440.  Layout under ``dataset_root``:
    ``CUB_200_2011/images/<rel_path>`` and ``CUB_200_2011/cachedir/cub/data/<split>_cub_cleaned.mat``
    (struct array ``images``: rel_path, bbox.{x1,y1,x2,y2} (1-based), parts (3 × 15: x, y, vis,
    1-based), mask) plus ``.../sfm/anno_<split>.mat`` (``sfm_anno``: scale, trans, rot).  Random
    draws (bbox jitter, mirror) come from ``np.random`` like the reference's, or from ``rng``."""

    def __init__(self, img_size=512, split="train", unsup_mask=False, dataset_root="~", single_class=None, rng=None):
        import scipy.io as sio
        self.img_size, self.split, self.unsup_mask = img_size, split, unsup_mask
        self.rng = rng if rng is not None else np.random
        root = os.path.join(os.path.expanduser(dataset_root), "CUB_200_2011")
        self.img_dir = os.path.join(root, "images")
        self.pmask_dir = os.path.join(os.path.expanduser(dataset_root), "pseudolabels")
        cache = os.path.join(root, "cachedir", "cub")
        anno_path = os.path.join(cache, "data", f"{split}_cub_cleaned.mat")
        if not os.path.exists(anno_path):
            raise FileNotFoundError(f"{anno_path} does not exist")
        self.anno = np.atleast_1d(sio.loadmat(anno_path, struct_as_record=False, squeeze_me=True)["images"])
        self.anno_sfm = np.atleast_1d(sio.loadmat(os.path.join(cache, "sfm", f"anno_{split}.mat"),
                                                  struct_as_record=False, squeeze_me=True)["sfm_anno"])
        self.labels = [int(str(a.rel_path).split(".")[0]) for a in self.anno]
        if single_class is not None:
            idx = [i for i, c in enumerate(self.labels) if c == single_class]
            self.anno = [self.anno[i] for i in idx]
            self.anno_sfm = [self.anno_sfm[i] for i in idx]
            self.labels = [self.labels[i] for i in idx]

    def __len__(self):
        return len(self.anno)

    def _forward_img(self, index):   # cub_parts.py:288-351
        from PIL import Image
        data, sfm = self.anno[index], self.anno_sfm[index]
        sfm_pose = [np.copy(sfm.scale), np.copy(sfm.trans).astype(np.float64), np.copy(sfm.rot)]
        rot = np.pad(sfm_pose[2], (0, 1), "constant")
        rot[3, 3] = 1
        sfm_pose[2] = _quaternion_from_rotation(rot)
        img_path = os.path.join(self.img_dir, str(data.rel_path))
        img = np.array(Image.open(img_path))
        if img.ndim == 2:   # grayscale
            img = np.repeat(img[:, :, None], 3, axis=2)
        if self.unsup_mask and self.split != "train":
            pm = Image.open(os.path.join(self.pmask_dir, str(data.rel_path).replace(".jpg", ".png")))
            mask = _resize_nearest(np.array(pm), img.shape[0], img.shape[1]) / 255.0
        else:
            mask = np.asarray(data.mask)
        mask = np.expand_dims(mask, 2)
        bbox = np.array([data.bbox.x1, data.bbox.y1, data.bbox.x2, data.bbox.y2], float) - 1
        kp = np.copy(np.asarray(data.parts).T.astype(float))
        vis = kp[:, 2] > 0
        kp[vis, :2] -= 1
        jf = CUB_JITTER_FRAC if self.split == "train" else 0
        bbox = _square_bbox(_perturb_bbox(bbox, CUB_PADDING_FRAC, jf, self.rng))
        # crop (cub_parts.py:365-373)
        img = _crop(img, bbox, bgval=1)
        mask = _crop(mask, bbox, bgval=0)
        kp[vis, 0] -= bbox[0]
        kp[vis, 1] -= bbox[1]
        sfm_pose[1][0] -= bbox[0]
        sfm_pose[1][1] -= bbox[1]
        # scale so the longer side is img_size (cub_parts.py:375-390)
        scale = self.img_size / float(max(img.shape[0], img.shape[1]))
        nh, nw = (np.round(np.array(img.shape[:2]) * scale)).astype(int)
        img = _resize_linear(img, nh, nw)
        mask = _resize_nearest(mask[:, :, 0] if mask.ndim == 3 else mask, nh, nw)
        kp[vis, :2] *= scale
        sfm_pose[0] = sfm_pose[0] * scale
        sfm_pose[1] = sfm_pose[1] * scale
        if self.split == "train" and self.rng.random() > 0.5:   # mirror (cub_parts.py:392-412); one draw, as rand(1)
            img = img[:, ::-1, :].copy()
            mask = mask[:, ::-1].copy()
            new_x = img.shape[1] - kp[:, 0] - 1
            kp = np.hstack((new_x[:, None], kp[:, 1:]))[CUB_KP_PERM, :]
            R = _quaternion_matrix(sfm_pose[2])
            flip = np.diag([-1, 1, 1, 1])
            sfm_pose[2] = _quaternion_from_rotation(flip.dot(R.dot(flip)))
            sfm_pose[1][0] = img.shape[1] - sfm_pose[1][0] - 1
        # normalise kp to [-1, 1] (cub_parts.py:353-363)
        h, w = img.shape[:2]
        v = kp[:, 2, None] > 0
        kp = v * np.stack([2 * (kp[:, 0] / w) - 1, 2 * (kp[:, 1] / h) - 1, kp[:, 2]]).T
        sfm_pose[0] = sfm_pose[0] * (1.0 / w + 1.0 / h)
        sfm_pose[1][0] = 2.0 * (sfm_pose[1][0] / w) - 1
        sfm_pose[1][1] = 2.0 * (sfm_pose[1][1] / h) - 1
        img_u8 = np.asarray(img, np.uint8)   # float64 -> uint8 truncation, as Image.fromarray(np.asarray(., uint8))
        return img_u8, kp, np.asarray(mask, np.float32), sfm_pose, img_path

    def __getitem__(self, index):   # cub_parts.py:417-440
        img, kp, mask, sfm_pose, img_path = self._forward_img(index)
        kpts = ((kp[:, :2] + 1) / 2)[:, [1, 0]]   # (row, col) in [0, 1]
        return {
            "img": torch.from_numpy(img.transpose(2, 0, 1).copy()).float() / 255.0,
            "kpts": torch.tensor(kpts),
            "visibility": torch.tensor(kp[:, 2]),
            "mask": np.expand_dims(mask, 2),
            "sfm_pose": np.concatenate([np.atleast_1d(sfm_pose[0]), sfm_pose[1], sfm_pose[2]]),
            "inds": index,
            "label": self.labels[index],
            "img_path": img_path,
        }


CUB_CLASSES = {"cub_001": 1, "cub_002": 2, "cub_003": 3, "cub_all": None}


def make_dataset(name, loc="~", max_len=-1, validation=False, image_size=512, split="train"):
    if name in ("celeba_aligned", "celeba_wild"):
        return CelebA(max_len=max_len, split=split, align=(name == "celeba_aligned"), dataset_loc=loc)
    if name in CUB_CLASSES:
        return CUBParts(split=split, dataset_root=loc, single_class=CUB_CLASSES[name])
    if name == "custom":
        ds = CustomDataset(loc, image_size)
    elif name == "synthetic":
        ds = SyntheticDataset(n=max_len if max_len > 0 else 64, size=image_size)
    else:
        raise NotImplementedError(f"dataset '{name}': readers built here are celeba_aligned, celeba_wild, cub_001, "
                                  "cub_002, cub_003, cub_all, custom and synthetic (or pass dataset=...)")
    if max_len > 0 and name == "custom":
        ds = torch.utils.data.Subset(ds, range(min(max_len, len(ds))))
    return ds
