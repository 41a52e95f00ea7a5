"""DDIM scheduler subset used by the hot path (diffusers-0.8.0 semantics).

Reference: ``optimize_token.load_ldm`` builds ``DDIMScheduler(beta_start=0.00085,
beta_end=0.012, beta_schedule="scaled_linear", clip_sample=False,
set_alpha_to_one=False)`` and calls ``set_timesteps(50)``
(``unsupervised_keypoints/optimize_token.py:25-35``); the hot path only uses
``timesteps`` and ``add_noise`` (``ptp_utils.py:219-229``).
"""
import numpy as np
import torch


class DDIMScheduler:
    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012,
                 beta_schedule="scaled_linear", clip_sample=False, set_alpha_to_one=False, steps_offset=0):
        if beta_schedule != "scaled_linear":
            raise NotImplementedError(beta_schedule)
        self.num_train_timesteps = num_train_timesteps
        self.betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.steps_offset = steps_offset
        self.timesteps = torch.from_numpy(np.arange(0, num_train_timesteps)[::-1].copy())

    def set_timesteps(self, num_inference_steps):
        ratio = self.num_train_timesteps // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64)
        self.timesteps = torch.from_numpy(ts + self.steps_offset)

    def _alphas_cumprod_on(self, device, dtype):
        """alphas_cumprod on the samples' device, uploaded once: a pageable host-to-device copy per
        call waits for everything queued on the stream (hipMemcpyWithStream), which stalled the host
        — and with it the GPU queue — at every capture."""
        cache = self.__dict__.setdefault("_ac_cache", {})
        key = (str(device), dtype)
        if key not in cache:
            cache[key] = self.alphas_cumprod.to(device=device, dtype=dtype)
        return cache[key]

    def add_noise(self, original_samples, noise, timesteps):
        ac = self._alphas_cumprod_on(original_samples.device, original_samples.dtype)
        timesteps = timesteps.to(original_samples.device)
        # index_select, not ac[t]: a 0-d index tensor is read back to the host (a sync, and not
        # allowed inside a HIP graph capture)
        a = ac.index_select(0, timesteps.reshape(-1)).reshape(timesteps.shape)
        sqrt_a = a ** 0.5
        sqrt_1ma = (1 - a) ** 0.5
        while sqrt_a.dim() < original_samples.dim():
            sqrt_a = sqrt_a.unsqueeze(-1)
            sqrt_1ma = sqrt_1ma.unsqueeze(-1)
        return sqrt_a * original_samples + sqrt_1ma * noise
