"""Random affine warp with exact inverse (reference ``invertable_transform.py:6-92``).

The warp itself (affine_grid + grid_sample, bilinear, zeros, align_corners=False)
runs as the HIP kernel ``skp_affine_warp`` (with its adjoint for gradients);
theta is drawn on the host exactly as the reference draws it (``torch.rand`` on
the CPU generator, in the order angle, scale, tx, ty per sample), so seeded runs
reproduce the reference's augmentations.
"""
import math

import torch

from . import ops


def _upload(t, device):
    """Host θ to the device without blocking the host (pinned staging, async copy); a pageable
    copy waits for everything queued on the stream."""
    if t.device.type != "cpu" or torch.device(device).type == "cpu":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


class RandomAffineWithInverse:
    def __init__(self, degrees=0, scale=(1.0, 1.0), translate=(0.0, 0.0)):
        self.degrees = degrees
        self.scale = scale
        self.translate = translate
        self.last_params = {"theta": torch.eye(2, 3).unsqueeze(0)}

    def create_affine_matrix(self, angle, scale, translations_percent):
        """invertable_transform.py:22-36."""
        a = math.radians(angle)
        theta = torch.tensor([[math.cos(a), math.sin(a), translations_percent[0]],
                              [-math.sin(a), math.cos(a), translations_percent[1]]], dtype=torch.float)
        theta[:, :2] = theta[:, :2] * scale
        return theta.unsqueeze(0)

    def draw_theta(self, batch, generator=None):
        """invertable_transform.py:40-57 (same RNG calls, same order); ``generator``: a
        torch.Generator instead of the global CPU generator the reference uses."""
        thetas = []
        g = generator
        for _ in range(batch):
            angle = torch.rand(1, generator=g).item() * (2 * self.degrees) - self.degrees
            sf = torch.rand(1, generator=g).item() * (self.scale[1] - self.scale[0]) + self.scale[0]
            tp = (torch.rand(1, generator=g).item() * (2 * self.translate[0]) - self.translate[0],
                  torch.rand(1, generator=g).item() * (2 * self.translate[1]) - self.translate[1])
            thetas.append(self.create_affine_matrix(angle, sf, tp))
        return torch.cat(thetas, dim=0)

    def __call__(self, img_tensor, theta=None):
        if theta is None:
            theta = self.draw_theta(img_tensor.shape[0])
        self.last_params = {"theta": theta.detach().cpu().float()}
        return ops.affine_warp(img_tensor, _upload(theta.float(), img_tensor.device))

    def theta_inverse(self):
        """2×3 part of the 3×3 inverse of each stored theta (invertable_transform.py:77-84), with the
        reference's arithmetic: ``torch.inverse`` of the fp32 batch on the host CPU (its θ lives on
        the CPU: ``optimize.py:386``, ``eval.py:242``), so on any host it is bit-identical to the θ⁻¹
        the reference would hand to affine_grid there (MKL's LU rounds the last bit per CPU code
        path: tests/golden/theta_inv.npz was recorded on the build host)."""
        theta = self.last_params["theta"].float()
        aug = torch.cat([theta, torch.tensor([[[0.0, 0.0, 1.0]]], dtype=torch.float32).expand(theta.shape[0], -1, -1)],
                        dim=1)
        return torch.inverse(aug)[:, :2, :].contiguous()

    def inverse(self, img_tensor):
        """invertable_transform.py:72-92: warp by the inverse of the stored thetas."""
        th = self.theta_inverse()
        if th.shape[0] != img_tensor.shape[0]:
            raise ValueError(f"inverse: {img_tensor.shape[0]} images but {th.shape[0]} stored thetas")
        return ops.affine_warp(img_tensor, _upload(th, img_tensor.device))
