"""HIP-graph replay of the token-optimisation pass (TokenOptimizer(graph=True)) vs the eager pass.

The graph pass (optimize.TokenOptimizer._graph_pass) runs the first prefetched pass eagerly,
captures the same pass into one torch.cuda.CUDAGraph and replays it for every later pass with the
new latents and inverse warps copied into its static inputs.  It must give what the eager
micro_steps gives (reference optimize.py:362-445: per-image selection, losses, the summed context
gradient and the Adam step): the same selected indices, the same running losses, the same
accumulated gradient over several passes of one optimiser step and the same context after Adam.
The equivariance adjoint scatters with atomics, so gradients are compared at rtol 1e-4."""
import numpy as np
import pytest
import torch

import recipes

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def N(t):
    return t.detach().cpu().numpy()


def _run(graph, steps, eager_first=False):
    from stablekeypoints_amd.optimize import TokenOptimizer
    from stablekeypoints_amd.optimize_token import load_ldm
    from stablekeypoints_amd.sd import TINY_CONFIG, TINY_IMAGE
    lat = TINY_IMAGE // 8
    noise = torch.randn(4, 4, lat, lat, generator=torch.Generator().manual_seed(5)).to(DEV)
    ldm, ctls, _ = load_ldm(DEV, "tiny", feature_upsample_res=32, config=TINY_CONFIG)
    inner = ldm.scheduler

    class Sched:
        timesteps = inner.timesteps

        def add_noise(self, x, n, t):
            return inner.add_noise(x, noise, t)
    ldm.scheduler = Sched()
    ctx = torch.from_numpy(recipes.random_logits(61, (1, 16, 32))).to(DEV)
    opt = TokenOptimizer(ldm, ctls, ctx, top_k=4, furthest_point_num_samples=8, accum=4, device=DEV,
                         graph=graph)
    eye = torch.tensor([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0]])
    thetas = iter(torch.from_numpy(recipes.uniform(70 + i, (2, 2, 3), -0.1, 0.1)).float() + eye
                  for i in range(2 * steps))
    opt.transform.draw_theta = lambda batch: next(thetas)[:batch]
    out = []
    for s in range(steps):
        for p in range(2):                       # two passes of 2 images per optimiser step
            imgs = [torch.from_numpy(recipes.uniform(100 + 4 * s + 2 * p + i, (1, 3, TINY_IMAGE, TINY_IMAGE))).to(DEV)
                    for i in range(2)]
            if not (eager_first and s > 0 and p == 0):
                opt.prefetch(imgs)               # else: an eager (non-prefetched) pass
            idx = opt.micro_steps(imgs)
            out.append(("idx", [N(t) for t in idx]))
            out.append(("grad", N(opt.context.grad).copy()))
        rec = opt.optimizer_step()
        out.append(("loss", float(rec["loss"])))
        out.append(("ctx", N(opt.context).copy()))
    torch.cuda.synchronize()
    return out, opt


@pytest.mark.parametrize("eager_first", [False, True])
def test_graph_pass_equals_eager_pass(eager_first):
    """eager_first: from the second optimiser step on, the step's first pass is not prefetched
    (it runs eagerly) and its second is a graph replay, which must add to — not replace — the
    gradient the eager pass accumulated."""
    eager, _ = _run(False, 3 if eager_first else 2, eager_first)
    graphed, opt = _run(True, 3 if eager_first else 2, eager_first)
    assert opt._g is not None, "the graph path did not run"
    assert len(eager) == len(graphed)
    for (ka, a), (kb, b) in zip(eager, graphed):
        assert ka == kb
        if ka == "idx":
            for x, y in zip(a, b):
                assert np.array_equal(x, y)
        elif ka == "grad":
            assert np.allclose(a, b, rtol=1e-4, atol=1e-8), np.abs(a - b).max()
        elif ka == "loss":
            assert abs(a - b) <= 1e-5 * abs(a)
        else:
            assert np.allclose(a, b, rtol=1e-4, atol=1e-7)
