"""Dev probe: where the tiled capture forward differs from the one-row kernel (SKP_MAPS_TILE)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from test_gpu_parity import _capture_maps_abi  # noqa: E402

for (B, H, sizes, R, N) in [(1, 1, (16,), 128, 500), (1, 1, (32,), 128, 500), (1, 2, (16,), 128, 500), (1, 8, (16, 16, 16, 32), 128, 500)]:
    g = torch.Generator().manual_seed(1)
    zs = [(torch.randn(B * H, s * s, N, generator=g) * 3).cuda() for s in sizes]
    os.environ["SKP_MAPS_TILE"] = "0"
    m0, s0 = _capture_maps_abi(zs, list(sizes), B, H, R)
    for ty in ("2", "4"):
        os.environ["SKP_MAPS_TILE"] = ty
        m1, s1 = _capture_maps_abi(zs, list(sizes), B, H, R)
        bad = ~(m1 == m0)
        print(B, H, sizes, R, N, "ty", ty, "bad", int(bad.sum()), "nan", int(torch.isnan(m1).sum()), flush=True)
        if bad.any():
            idx = bad.nonzero()
            print("  tokens", idx[:, 1].unique()[:20].tolist())
            print("  rows", idx[:, 2].unique()[:40].tolist())
            print("  cols", idx[:, 3].unique()[:40].tolist())
            print("  sample", [(tuple(i.tolist()), m0[tuple(i)].item(), m1[tuple(i)].item()) for i in idx[:5]])
        sb = [int((~(a == b)).sum()) for a, b in zip(s1, s0)]
        print("  stats bad", sb)
