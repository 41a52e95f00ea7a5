"""GPU probe: fp32 SD-1.5 UNet / VAE-encoder timings on one MI355X (dev tool)."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from stablekeypoints_amd.sd import build_sd15, CrossAttention

def timeit(fn, n=3):
    torch.cuda.synchronize(); t0 = time.time(); fn(); torch.cuda.synchronize(); first = time.time() - t0
    ts = []
    for _ in range(n):
        torch.cuda.synchronize(); t0 = time.time(); fn(); torch.cuda.synchronize(); ts.append(time.time() - t0)
    return first, min(ts)

dev = "cuda:0"
t0 = time.time()
sd = build_sd15(device=dev)
print("build", time.time() - t0, flush=True)
print(torch.cuda.get_device_name(0), flush=True)
res = {}
for cl in (False, True):
    if cl:
        sd.unet.to(memory_format=torch.channels_last); sd.vae.to(memory_format=torch.channels_last)
    for B in (1, 2):
        img = torch.rand(B, 3, 512, 512, device=dev)
        if cl: img = img.contiguous(memory_format=torch.channels_last)
        def vae():
            with torch.no_grad():
                return sd.vae.encode(img * 2 - 1)["latent_dist"].mean
        res[f"vae_B{B}_cl{int(cl)}"] = timeit(vae); print(res, flush=True)
        lat = torch.randn(B, 4, 64, 64, device=dev)
        if cl: lat = lat.contiguous(memory_format=torch.channels_last)
        ctx = torch.randn(1, 500, 768, device=dev, requires_grad=True)
        for be in ("sdpa", "math"):
            CrossAttention.backend = be
            def fwd():
                with torch.no_grad():
                    return sd.unet(lat, sd.scheduler.timesteps[-1], ctx.repeat(B, 1, 1))["sample"]
            def fwdbwd():
                out = sd.unet(lat, sd.scheduler.timesteps[-1], ctx.repeat(B, 1, 1))["sample"]
                out.square().mean().backward()
            res[f"unet_fwd_B{B}_{be}_cl{int(cl)}"] = timeit(fwd)
            res[f"unet_fwdbwd_B{B}_{be}_cl{int(cl)}"] = timeit(fwdbwd)
            print(res, flush=True)
print(json.dumps(res, indent=1))
print("max mem GB", torch.cuda.max_memory_allocated() / 1e9)
