"""Map aggregation, losses and the token-optimisation loop (mirror of reference ``optimize.py``).

``optimize_embedding`` keeps the reference signature (``optimize.py:269-299``).
Parallelism is one process per GPU (``torch.distributed``, RCCL over xGMI)
instead of ``nn.DataParallel``: each rank runs the reference's per-replica body on
its own image, and the token-embedding gradient is all-reduced (SUM ÷ world)
once per optimiser step, which reproduces the reference's mean over replicas
(``optimize.py:428-443``).  See DESIGN.md §Multi-GPU.
"""
import json
import os
import time

import torch
import torch.nn.functional as F

from . import ops, ptp_utils
from . import eval as skp_eval
from .invertable_transform import RandomAffineWithInverse

# A/B: 0 = select per image (one top-k / FPS launch chain per image, r03ao and before)
SEL_BATCH = True


def _upload(t, device):
    """A small host tensor to the device without blocking the host: pinned staging + an async copy
    (a pageable copy is hipMemcpyWithStream, which waits for everything queued on the stream)."""
    if t.device.type != "cpu" or torch.device(device).type == "cpu":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


def collect_maps(controller, from_where=("up_cross",), upsample_res=512, layers=(0, 1, 2, 3), indices=None):
    """optimize.py:27-79: mean over the selected stored layers and B·heads -> (N', R', R').

    Runs ``skp_aggregate`` (+ ``skp_resize_bilinear``).  As in the reference the
    upsample guard compares the token count (optimize.py:63), i.e. it fires for any
    ``upsample_res != -1``; the bilinear resize is applied after the mean, which is
    equal because both are linear.
    """
    if getattr(controller, "stores_logits", False):
        # LogitStore: per-image fused maps, then the reference's mean over images (B·heads)
        R = getattr(controller, "feature_upsample_res", None)
        BH = controller.step_store["attn"][0].shape[0]
        H = controller.heads
        out = controller.maps_per_image(BH // H, R, layers).mean(dim=0)
        if indices is not None:
            out = out[torch.as_tensor(indices, device=out.device)]
        if upsample_res != -1 and upsample_res != out.shape[-1]:
            out = ops.resize_bilinear(out, upsample_res)
        controller.reset()
        return out
    attention_maps = controller.step_store["attn"]
    chosen = [a for li, a in enumerate(attention_maps) if li in layers]
    if not chosen:
        raise RuntimeError("collect_maps: no stored attention maps for layers %s" % (list(layers),))
    idx = None
    if indices is not None:
        idx = torch.as_tensor(indices, dtype=torch.int64)
    out = ops.aggregate(chosen, indices=idx, upsample_res=upsample_res)
    controller.reset()
    return out


def equivariance_loss(embeddings_initial, embeddings_transformed, transform, index):
    """optimize.py:157-163: mse(A, inverse(At)[index]) — only replica ``index``'s theta matters.

    ``embeddings_transformed`` is (replicas, T, h, w) or (T, h, w).
    """
    At = embeddings_transformed[index] if embeddings_transformed.dim() == 4 else embeddings_transformed
    th_inv = transform.theta_inverse()[int(index)]
    return ops.equivariance_loss_single(embeddings_initial, At, th_inv)


def sharpening_loss(attn_map, sigma=1.0, temperature=1e1, device="cuda", num_subjects=1):
    """optimize.py:166-179 (+ find_gaussian_loss_at_point 182-206): mse to Gaussians at the k-max pixels."""
    return ops.sharpening_loss(attn_map, sigma=sigma, num_subjects=num_subjects)


def find_gaussian_loss_at_point(attn_map, pos, sigma=1.0, temperature=1e-1, device="cuda", indices=None,
                                num_subjects=1):
    """optimize.py:182-206 with explicit positions pos (num, T, 2) in [0, 1]."""
    T, H, W = attn_map.shape
    target = ops.gaussian_circles(pos, H, sigma)
    if indices is not None:
        attn_map = attn_map[indices]
        target = target[indices]
    return F.mse_loss(attn_map, target)


def _make_dataset(dataset_name, dataset_loc, max_len, validation):
    from . import datasets
    return datasets.make_dataset(dataset_name, dataset_loc, max_len=max_len, validation=validation)


def _world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


class TokenOptimizer:
    """One rank's share of the token optimisation (optimize.py:337-471 loop body).

    ``micro_step(image)`` runs one reference micro-iteration on one image: capture
    on the image and on its random affine warp, top-k selection, furthest-point
    sampling, sharpening + equivariance losses, backward into ``context``.
    ``optimizer_step()`` all-reduces the gradient over ranks (SUM ÷ world) and
    applies Adam, as the reference does every ``batch_size // num_gpus`` micro-steps.
    """

    def __init__(self, ldm, controllers, context, lr=5e-3, top_k_strategy="gaussian", top_k=10,
                 furthest_point_num_samples=25, sigma=2.0, num_subjects=1, sharpening_loss_weight=100,
                 equivariance_attn_loss_weight=1000.0, accum=4, noise_level=-1, layers=(0, 1, 2, 3),
                 from_where=("down_cross", "mid_cross", "up_cross"), augment_degrees=15, augment_scale=(0.8, 1.0),
                 augment_translate=(0.25, 0.25), device="cuda", batch_captures=True, graph=False):
        self.ldm, self.controllers, self.device = ldm, controllers, device
        # graph: replay the prefetched-latents pass (capture forward, selection, losses, backward)
        # as ONE HIP graph (micro_steps); the host then issues one launch per pass instead of ~1500
        self.graph = graph
        # where micro_steps enqueues the next passes' VAE prefetch: "capture_bwd" = right after the
        # sparse capture backward, "bwd" = between the forward and the backward
        self.prefetch_at = "capture_bwd"
        self._g = None           # (key, HIPGraph, static inputs, static outputs) once captured
        self._grad_acc = None
        self._gstream = None
        # batch_captures: run each image with its warp in one VAE/UNet pass (micro_steps: all
        # of an optimiser step's images in one pass)
        # (run_and_find_attn_per_image); False = the reference's two sequential passes.
        self.batch_captures = batch_captures
        self._orig_controllers = controllers
        if batch_captures:
            # the fast path captures logits (LogitStore) and builds per-image maps fused
            R = getattr(ldm, "feature_upsample_res", 128)
            store = ptp_utils.LogitStore(early_exit=True)
            store.feature_upsample_res = R
            ptp_utils.register_attention_control(ldm.unet, store, feature_upsample_res=R)
            self.controllers = {k: store for k in controllers} if controllers else {torch.device(device): store}
        self.context = context
        self.context.requires_grad = True
        self.optimizer = torch.optim.Adam([self.context], lr=lr)
        self.top_k_strategy, self.top_k, self.fps_n = top_k_strategy, top_k, furthest_point_num_samples
        self.sigma, self.num_subjects = sigma, num_subjects
        self.w_sharp, self.w_eq = sharpening_loss_weight, equivariance_attn_loss_weight
        self.accum = accum
        self.kw = dict(layers=layers, noise_level=noise_level, from_where=from_where, upsample_res=-1, device=device,
                       controllers=controllers)
        self.transform = RandomAffineWithInverse(degrees=augment_degrees, scale=augment_scale,
                                                 translate=augment_translate)
        self.world, self.rank = _world()
        if self.world > 1:
            # every rank must start from rank 0's embedding: the ranks apply identical Adam
            # steps to identical all-reduced gradients, so one broadcast keeps them in lockstep
            import torch.distributed as dist
            with torch.no_grad():
                dist.broadcast(self.context, src=0)
            self.sync_cpu_rng()
        self._prefetched = []      # FIFO of (key, thetas, latents, event) from prefetch()
        self._side = None
        self.reset_running()

    def prefetch(self, images):
        """Warp and VAE-encode an optimiser step's images (and draw their thetas) ahead of time
        on a side stream, so the VAE encoder — a third of the step, independent of the
        context — overlaps the previous step's UNet backward.  The thetas are drawn here, in the
        same order as ``micro_steps`` would draw them; ``micro_steps(images)`` then consumes
        the record.  A no-op for images already prefetched or without ``batch_captures``."""
        key = tuple(id(t) for t in images)
        if not self.batch_captures or any(r[0] == key for r in self._prefetched):
            return
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        batch = torch.cat(list(images))
        thetas = self.draw_thetas(len(images))
        main = torch.cuda.current_stream(self.device)
        self._side.wait_stream(main)
        with torch.cuda.stream(self._side), torch.no_grad():
            batch.record_stream(self._side)
            transformed = ops.affine_warp(batch, _upload(thetas.float(), self.device))
            lat = ptp_utils.image2latent(self.ldm, torch.cat([batch, transformed]), self.device)
            ev = torch.cuda.Event()
            ev.record(self._side)
        self._prefetched.append((key, thetas, lat, ev))

    def draw_thetas(self, k):
        """Warps for this rank's next ``k`` micro-iterations, drawn as the reference draws them.

        The reference applies the transform to each micro-iteration's DataParallel batch of
        ``num_gpus`` images (optimize.py:386), so its CPU generator yields, per micro-iteration,
        one theta per replica in replica order; replica r uses theta r (optimize.py:420-424).
        Every rank draws the whole sequence (k·world thetas, same CPU seed on every rank) and keeps
        its own column, so the run is the same augmentation stream at any world size.  The ranks'
        CPU generators agree because ``sync_cpu_rng`` copies rank 0's into every rank when the
        optimiser is built."""
        if self.world == 1:
            return self.transform.draw_theta(k)
        th = self.transform.draw_theta(k * self.world)
        return th.reshape(k, self.world, 2, 3)[:, self.rank].contiguous()

    def sync_cpu_rng(self):
        """Give every rank rank 0's CPU generator state (world > 1).  The reference is one process
        with one CPU generator, which draws every replica's warp (optimize.py:386); here each rank
        draws the whole replica-ordered sequence and keeps its column (``draw_thetas``), which is
        the reference's stream only if the ranks' generators agree — whatever seeds the caller
        gave each rank."""
        import torch.distributed as dist
        state = torch.get_rng_state()
        if dist.get_backend() == "nccl":
            state = state.to(self.context.device)
        dist.broadcast(state, src=0)
        torch.set_rng_state(state.cpu())

    def _take_prefetched(self, images):
        key = tuple(id(t) for t in images)
        if self._prefetched and self._prefetched[0][0] == key:
            _, thetas, lat, ev = self._prefetched.pop(0)
            main = torch.cuda.current_stream(self.device)
            main.wait_event(ev)
            lat.record_stream(main)
            return thetas, lat
        return None

    def restore_hooks(self):
        """Point the patched attention back at the caller's controllers."""
        if self.batch_captures and self._orig_controllers:
            ctl = next(iter(self._orig_controllers.values()))
            R = getattr(self.ldm, "feature_upsample_res", 128)
            ptp_utils.register_attention_control(self.ldm.unet, ctl, feature_upsample_res=R)

    def reset_running(self):
        self.run_eq = self.run_sh = self.run_tot = 0.0

    def micro_step(self, image):
        """One reference micro-iteration on ``image`` (1, 3, H, W): loss, backward, running stats."""
        loss, eq, sh, idx = self.image_loss(image)
        self._account(loss, eq, sh)
        (loss / self.accum).backward()
        return idx

    def _account(self, loss, eq, sh):
        self.run_eq = self.run_eq + eq.detach() / self.accum * self.w_eq
        self.run_sh = self.run_sh + sh.detach() / self.accum * self.w_sharp
        self.run_tot = self.run_tot + loss.detach() / self.accum

    def micro_steps(self, images, prefetch=()):
        """``len(images)`` reference micro-iterations in ONE VAE/UNet pass of batch 2·k (every
        image and its warp) and ONE backward.

        The micro-iterations of an optimiser step are independent given the shared context
        (optimize.py:362-445 sums their gradients before Adam), so this equals k ``micro_step``
        calls up to fp32 summation order: the thetas are drawn in the same order from the CPU
        generator, and the selection and losses stay per image.  A batch of 2·k images fills
        the 256 CUs far better than k passes of 2 (the UNet's 64²-and-smaller convolutions and
        GEMMs are too small at batch 2).  Returns the per-image selected token indices.
        ``prefetch``: image batches whose VAE encoding (``prefetch``) is enqueued on the side stream
        between this pass's forward and its backward — the host issues those ~130 launches while
        the main stream still works through the queued forward; issued after the backward they
        left the main stream idle before Adam (≈7 ms per step, tools/stream_gaps.py).
        """
        if not self.batch_captures or len(images) == 1:
            return [self.micro_step(img) for img in images]
        k = len(images)
        pre = self._take_prefetched(images)
        if pre is not None and self.graph and ops.SEL_BWD:
            thetas, inputs = pre
            self.transform.last_params = {"theta": thetas.detach().cpu().float()}
            return self._graph_pass(k, inputs, prefetch)
        if pre is not None:                              # latents of images + warps (prefetch)
            thetas, inputs = pre
            self.transform.last_params = {"theta": thetas.detach().cpu().float()}
        else:
            batch = torch.cat(list(images))
            transformed = self.transform(batch, theta=self.draw_thetas(k))   # k thetas, image order
            inputs = torch.cat([batch, transformed])
        sparse = ops.SEL_BWD
        got = ptp_utils.run_and_find_attn_per_image(
            self.ldm, inputs, self.context, noise_level=self.kw["noise_level"], device=self.device,
            layers=self.kw["layers"], controllers=self.controllers, stacked=True, captured=sparse)[0]
        maps = got.maps if sparse else got        # (2k, N, R, R); the selection needs no gradient
        th_inv = _upload(self.transform.theta_inverse(), self.device)   # all k warps, one upload
        sel = self._select_batch(maps[:k], maps[k:])
        if sparse:
            # every image's selected rows in ONE gather whose backward is the sparse capture backward
            # (skp_capture_maps_bwd_sel): the rows' gradient goes straight to the kernel, no
            # (2k, N, R, R) map gradient is formed
            rows = got.select(sel + sel)
            n = rows.shape[0] // 2
            A, At = rows[:n], rows[n:]
        else:
            # one gather of every image's selected rows (its backward is one scatter into the
            # (2k, N, R, R) map gradient instead of 2k full-size zero-fills and adds)
            img = torch.cat([torch.full_like(idx, i) for i, idx in enumerate(sel)])
            tok = torch.cat(sel)
            A, At = maps[img, tok], maps[img + k, tok]
        total, parts = self._pass_losses(sel, A, At, th_inv)
        for loss, eq, sh in parts:
            self._account(loss, eq, sh)
        if sparse and prefetch and self.prefetch_at == "capture_bwd":
            # the next passes' VAE enqueued right behind the sparse capture backward (select()'s
            # backward calls it): the VAE then shares the GPU with the UNet backward's GEMMs and
            # convolutions rather than with the capture backward's VALU kernels
            got.after_backward = lambda: [self.prefetch(b) for b in prefetch]
            (total / self.accum).backward()
            if got.after_backward is not None:    # the hook did not run (no selected rows)
                got.after_backward()
                got.after_backward = None
            return sel
        for b in prefetch:
            self.prefetch(b)
        (total / self.accum).backward()
        return sel

    def _pass_body(self, k, inputs, th_inv):
        """The prefetched-latents pass of micro_steps (sparse backward path): capture, selection,
        losses, backward.  Returns (selected indices per image, (loss, eq, sh) per image)."""
        got = ptp_utils.run_and_find_attn_per_image(
            self.ldm, inputs, self.context, noise_level=self.kw["noise_level"], device=self.device,
            layers=self.kw["layers"], controllers=self.controllers, stacked=True, captured=True)[0]
        maps = got.maps
        sel = self._select_batch(maps[:k], maps[k:])
        rows = got.select(sel + sel)
        n = rows.shape[0] // 2
        A, At = rows[:n], rows[n:]
        total, parts = self._pass_losses(sel, A, At, th_inv)
        (total / self.accum).backward()
        return sel, parts

    def _graph_pass(self, k, inputs, prefetch):
        """micro_steps as a replay of ONE captured HIP graph.

        The pass has static shapes (k images + warps, N tokens, fixed top-k / FPS counts), so its
        ~1500 kernels are captured once (torch.cuda.graph: the UNet/VAE GEMMs, MIOpen, and every
        libskp launch, which all go to the current stream) and replayed with the new latents and
        inverse warps copied into the graph's static inputs; the noise draw advances the CUDA
        generator's offset per replay as in eager execution.  The first call runs the pass eagerly
        (that step's real work) and then captures it; the gradient the graph writes is added to
        this optimiser step's accumulator, so several passes per step still sum as in eager mode.
        Same kernels and arithmetic as the eager pass (tests/test_gpu_graph.py)."""
        th_inv = _upload(self.transform.theta_inverse(), self.device)
        for b in prefetch:                      # the next passes' VAE, before this pass is issued
            self.prefetch(b)
        key = (tuple(inputs.shape), tuple(th_inv.shape))
        if self._g is None or self._g[0] != key:
            # eager pass (this step's work) on the capture stream — the warm-up torch's graph capture
            # wants on the stream it captures on — then the same pass captured into a graph
            main = torch.cuda.current_stream(self.device)
            if self._gstream is None:
                self._gstream = torch.cuda.Stream(device=self.device)
            side = self._gstream
            side.wait_stream(main)
            inputs.record_stream(side)
            th_inv.record_stream(side)
            prev = self.context.grad
            self.context.grad = None
            with torch.cuda.stream(side):
                sel, parts = self._pass_body(k, inputs, th_inv)
                eager_grad = self.context.grad
                s_in, s_th = inputs.clone(), th_inv.clone()
            g = torch.cuda.CUDAGraph()
            self.context.grad = None
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, stream=side):
                    s_sel, s_parts = self._pass_body(k, s_in, s_th)
            main.wait_stream(side)
            self._g = (key, g, (s_in, s_th), (s_sel, s_parts, self.context.grad))
            grad = eager_grad
        else:
            _, g, (s_in, s_th), (s_sel, s_parts, s_grad) = self._g
            prev = self.context.grad     # eager passes of this step too (zero_grad leaves None)
            s_in.copy_(inputs)
            s_th.copy_(th_inv)
            g.replay()
            sel = [x.clone() for x in s_sel]
            parts = [tuple(x.clone() for x in p) for p in s_parts]
            grad = s_grad
        # this step's gradient: the pass's, plus what earlier passes of the step accumulated
        self._grad_acc = grad.clone() if prev is None else prev + grad
        self.context.grad = self._grad_acc
        for loss, eq, sh in parts:
            self._account(loss, eq, sh)
        return sel

    def image_loss(self, image):
        """optimize.py:372-437 for one image: (weighted loss, equivariance, sharpening, indices)."""
        if self.batch_captures:
            transformed_img = self.transform(image, theta=self.draw_thetas(1))
            attn_map, attention_map_transformed = ptp_utils.run_and_find_attn_per_image(
                self.ldm, torch.cat([image, transformed_img]), self.context, noise_level=self.kw["noise_level"],
                device=self.device, layers=self.kw["layers"], controllers=self.controllers)[0]
        else:
            attn_map = ptp_utils.run_and_find_attn(self.ldm, image, self.context, **self.kw)[0]
            transformed_img = self.transform(image, theta=self.draw_thetas(1))
            attention_map_transformed = ptp_utils.run_and_find_attn(self.ldm, transformed_img, self.context,
                                                                     **self.kw)[0]
        return self._map_loss(attn_map, attention_map_transformed, 0)

    def _map_loss(self, attn_map, attention_map_transformed, index):
        """optimize.py:403-437 for one image's maps; ``index`` selects its theta in ``self.transform``."""
        idx = self._select(attn_map, attention_map_transformed)
        loss, eq, sh = self._losses(attn_map[idx], attention_map_transformed[idx], index)
        return loss, eq, sh, idx

    def _select_batch(self, maps, maps_t):
        """_select for k images at once: maps / maps_t (k, N, R, R) = the images' and their warps'
        maps.  The Gaussian KL keys, the candidates' ranking + argmax, and the furthest-point
        sampling run as one launch each over the k images (ops.gaussian_fps_batch); each image's
        selection is the reference's for that image (optimize.py:403-424 per replica).  Falls back to per-image
        _select where the batched form does not apply (other strategies, fewer candidates than
        top_k)."""
        k, N = maps.shape[0], maps.shape[1]
        n_cand = min(int(self.fps_n), N)
        if not (SEL_BATCH and k > 1 and self.top_k_strategy == "gaussian" and 2 <= self.top_k <= n_cand):
            return [self._select(maps[i], maps_t[i]) for i in range(k)]
        # KL keys → (ranking + the candidates' argmax on the warps' maps) → FPS: three launches
        sel, _, _ = ops.gaussian_fps_batch(maps, maps_t, n_cand, self.top_k, sigma=self.sigma,
                                           num_subjects=self.num_subjects)
        return list(sel.unbind(0))

    def _select(self, attn_map, attention_map_transformed):
        """optimize.py:403-424: top-k candidates on the image's map, FPS on its warp's map."""
        if self.top_k_strategy == "entropy":
            cand = ptp_utils.entropy_sort(attn_map, self.fps_n)
        elif self.top_k_strategy == "gaussian":
            cand = ptp_utils.find_top_k_gaussian(attn_map, self.fps_n, sigma=self.sigma, num_subjects=self.num_subjects)
        elif self.top_k_strategy == "consistent":
            cand = torch.arange(self.fps_n, device=attn_map.device)
        else:
            raise NotImplementedError
        return ptp_utils.furthest_point_sampling(attention_map_transformed, self.top_k, cand)

    def _pass_losses(self, sel, A, At, th_inv):
        """The losses of every image of a pass (optimize.py:425-437 per replica) on the stacked
        selected rows A / At (image i's rows follow image i−1's).  Returns (the pass's total,
        [(loss, eq, sh)] to account).  With equal row counts the sharpening and equivariance
        losses of all images run as one launch each per direction (ops.*_loss_batch: each
        image's loss and gradient are the per-image call's); the accounted statistics are then
        the pass's sums."""
        k = len(sel)
        n = sel[0].numel() if k else 0
        if SEL_BATCH and k > 1 and all(t.numel() == n for t in sel) and A.shape[0] == k * n:
            sh = ops.sharpening_loss_batch(A, k, sigma=self.sigma, num_subjects=self.num_subjects)
            eq = ops.equivariance_loss_batch(A, At, th_inv[:k], k)
            loss = eq * self.w_eq + sh * self.w_sharp
            total = loss.sum()
            return total, [(total, eq.sum(), sh.sum())]
        total, off, parts = 0.0, 0, []
        for i, idx in enumerate(sel):
            m = idx.numel()
            loss, eq, sh = self._losses(A[off:off + m], At[off:off + m], i, th_inv[i])
            off += m
            parts.append((loss, eq, sh))
            total = total + loss
        return total, parts

    def _losses(self, A, At, index, theta_inv=None):
        """optimize.py:425-437 on the selected rows; ``index`` selects the warp's theta
        (``theta_inv``: that theta's inverse already on the device)."""
        sh = sharpening_loss(A, device=self.device, sigma=self.sigma, num_subjects=self.num_subjects)
        if theta_inv is not None:
            eq = ops.equivariance_loss_single(A, At, theta_inv)
        else:
            eq = equivariance_loss(A, At, self.transform, index)   # (T, h, w): theta ``index``
        loss = eq * self.w_eq + sh * self.w_sharp
        return loss, eq, sh

    def optimizer_step(self):
        if self.world > 1:
            # ONE all-reduce per optimiser step: the embedding gradient and the three loss statistics
            # in one flat buffer (SUM, then ÷ world: the reference's mean over replicas,
            # optimize.py:428-443)
            import torch.distributed as dist
            g = self.context.grad
            stats = torch.stack([torch.as_tensor(x, device=g.device, dtype=g.dtype).reshape(())
                                 for x in (self.run_tot, self.run_eq, self.run_sh)])
            flat = torch.cat([g.reshape(-1), stats])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM)
            flat.div_(self.world)
            g.copy_(flat[:g.numel()].view_as(g))
            self.run_tot, self.run_eq, self.run_sh = flat[g.numel():].unbind(0)
        self.optimizer.step()
        self.optimizer.zero_grad()
        self._grad_acc = None
        rec = {"loss": self.run_tot, "running_equivariance_attn_loss": self.run_eq,
               "running_sharpening_loss": self.run_sh}
        self.reset_running()
        return rec


class ReplicaSampler:
    """The reference's ``DataLoader(dataset, batch_size=num_gpus, shuffle=True, drop_last=True)``
    (optimize.py:356-368) split over ranks: each epoch is one permutation shared by every rank
    (one seed, broadcast from rank 0 when not given), cut into groups of ``num_gpus`` with the
    remainder dropped; micro-iteration j gives rank r element r of group j, i.e. exactly the image
    DataParallel replica r receives.  The ranks' images are therefore a partition of each group."""

    def __init__(self, n, num_gpus, rank, seed=None):
        if n < num_gpus:
            raise ValueError(f"dataset of {n} images cannot fill a group of num_gpus={num_gpus} (drop_last)")
        if seed is None:
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,)))
            if num_gpus > 1:
                import torch.distributed as dist
                t = torch.tensor([seed], dtype=torch.int64)
                if dist.get_backend() == "nccl":
                    t = t.cuda()
                dist.broadcast(t, src=0)
                seed = int(t.item())
        self.n, self.g, self.rank = n, num_gpus, rank
        self.gen = torch.Generator().manual_seed(int(seed))
        self.groups = 0
        self.pos = 0

    def next(self):
        if self.pos >= self.groups:
            self.order = torch.randperm(self.n, generator=self.gen)
            self.groups = self.n // self.g
            self.pos = 0
        i = int(self.order[self.pos * self.g + self.rank])
        self.pos += 1
        return i


def optimize_embedding(ldm, top_k_strategy="entropy", wandb_log=True, context=None, device="cuda", num_steps=2000,
                       from_where=("down_cross", "mid_cross", "up_cross"), upsample_res=256, layers=(0, 1, 2, 3, 4, 5),
                       lr=5e-3, noise_level=-1, num_tokens=1000, top_k=10, augment_degrees=30,
                       augment_scale=(0.9, 1.1), augment_translate=(0.1, 0.1), dataset_loc="~", sigma=1.0,
                       sharpening_loss_weight=100, equivariance_attn_loss_weight=100, batch_size=4, num_gpus=1,
                       dataset_name="celeba_aligned", max_len=-1, min_dist=0.05, furthest_point_num_samples=50,
                       controllers=None, validation=False, num_subjects=1, dataset=None, log=None, seed=None):
    """optimize.py:269-475.  Extra keyword conveniences: ``dataset`` (object yielding
    {"img": (3,H,W)}; overrides dataset_name), ``log`` (callable receiving each
    optimiser step's metrics instead of print), ``seed`` (shuffle seed, the same on every rank;
    default: drawn on rank 0 and broadcast).  Rank r processes replica r's images
    (``ReplicaSampler``) with replica r's warps (``TokenOptimizer.draw_thetas``)."""
    world, rank = _world()
    num_gpus = world   # one process per GPU: the replica count is the world size
    if dataset is None:
        dataset = _make_dataset(dataset_name, dataset_loc, max_len, validation)
    if context is None:
        context = ptp_utils.init_random_noise(device, num_words=num_tokens,
                                              dim=getattr(ldm.unet, "cross_attention_dim", 768))
    accum = batch_size // num_gpus
    opt = TokenOptimizer(ldm, controllers, context, lr=lr, top_k_strategy=top_k_strategy, top_k=top_k,
                         furthest_point_num_samples=furthest_point_num_samples, sigma=sigma,
                         num_subjects=num_subjects, sharpening_loss_weight=sharpening_loss_weight,
                         equivariance_attn_loss_weight=equivariance_attn_loss_weight, accum=max(accum, 1),
                         noise_level=noise_level, layers=layers, from_where=from_where,
                         augment_degrees=augment_degrees, augment_scale=augment_scale,
                         augment_translate=augment_translate, device=device)
    n_iter = int(num_steps * accum)   # batch_size < num_gpus gives 0 iterations, as in the reference
    sampler = ReplicaSampler(len(dataset), num_gpus, rank, seed)

    def next_image():
        return dataset[sampler.next()]["img"][None].to(device, non_blocking=True)

    def next_batch(n):
        return [next_image() for _ in range(n)]

    start = time.time()
    it_start = time.time()
    done = 0
    cur = next_batch(min(accum, n_iter)) if n_iter > 0 else []
    while done < n_iter:
        n = len(cur)
        nxt = next_batch(min(accum, n_iter - done - n)) if done + n < n_iter else []
        opt.prefetch(cur)                 # no-op when already prefetched
        if nxt:
            opt.prefetch(nxt)             # the next step's VAE pass overlaps this step's UNet pass
        opt.micro_steps(cur)              # the optimiser step's images in one VAE/UNet pass
        done += n
        if done % accum == 0:
            rec = {k: float(v) for k, v in opt.optimizer_step().items()}
            rec["iteration time"] = time.time() - it_start
            if log is not None:
                log(rec)
            elif rank == 0:
                print(json.dumps(rec) if wandb_log else
                      f"loss: {rec['loss']}, _loss_equivariance_attn: {rec['running_equivariance_attn_loss']} "
                      f"sharpening_loss: {rec['running_sharpening_loss']}, iteration time: {rec['iteration time']}",
                      flush=True)
            it_start = time.time()
        cur = nxt
    opt.restore_hooks()
    if rank == 0 and log is None:
        print(f"optimization took {time.time() - start} seconds", flush=True)
    return context.detach()
