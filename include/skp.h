/*
 * skp.h — C ABI of libskp.so, the MI355X (gfx950) hot path of StableKeypoints.
 *
 * The reference (damaggu/StableKeypoints) has no FFI: its hot path is Python/torch
 * (SURVEY.md §8b).  Each entry point below replaces one reference function or the
 * torch-op sequence inside it; the reference file:line is cited per function.
 * The Python mirror of the reference API (stablekeypoints_amd/) binds these with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - All pointers are DEVICE pointers to row-major fp32 / int64 buffers that the
 *     caller allocates (caller owns every buffer; the library keeps no global state
 *     and is safe to call concurrently on different streams).
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *   - Return 0 on success, SKP_EBADARG (-1) for invalid arguments, SKP_ELAUNCH (-2)
 *     when a kernel launch fails.  skp_last_error() gives the thread-local message.
 *   - "maps" are (T, h, w) fp32; "positions" are (row + 0.5, col + 0.5) fp32 pairs;
 *     "attn" is one captured layer (BH, R*R, N) fp32 in the reference layout
 *     (ptp_utils.py:534-536: (batch*heads, pixels, tokens)).
 */
#ifndef SKP_H
#define SKP_H

#ifdef __cplusplus
extern "C" {
#endif

#define SKP_OK 0
#define SKP_EBADARG (-1)
#define SKP_ELAUNCH (-2)
#define SKP_MAX_LAYERS 16

const char* skp_last_error(void);
int skp_version(void);

/* ---------------------------------------------------------------- A1 capture
 * Replaces the capture branch of the patched CrossAttention.forward,
 * ptp_utils.py:508-538 (bicubic(x) -> to_q -> q kᵀ·scale -> softmax).  With
 * z_low = the layer's normal-path logits q kᵀ·scale at s×s (ptp_utils.py:493),
 * attn[b,p,n] = softmax_n(bicubic_{s->R}(z_low[b,:,n])[p]).
 *   z_low (BH, s*s, N) -> attn (BH, R*R, N).  `stats` (may be NULL): (BH, R*R, 2) floats
 *   receive each pixel's softmax row max and 1/Σexp, which the backward can reuse.     */
int skp_capture_fwd(const float* z_low, int BH, int s, int N, int R, float* attn, float* stats, void* stream);

/* Backward of skp_capture_fwd: dz_low = bicubicᵀ( a ⊙ (g − Σ_n a g) ), g = gscale·dattn.
 * Row b of g starts at dattn + (b / group)·sb and is read with strides (sp, sn), so a
 * broadcast gradient needs no materialisation: the layer/head mean of collect_maps gives
 * group = BH, sb = 0; a per-image map gradient (B, N, R²) gives group = heads,
 * sb = N·R², sp = 1, sn = R².  `workspace` holds BH*R*s*N floats (row-adjoint partials).
 * `stats`: the forward's per-pixel (max, 1/Σ) or NULL (recomputed by two row reductions). */
int skp_capture_bwd(const float* z_low, int BH, int s, int N, int R, const float* dattn, int group, long long sb,
                    long long sp, long long sn, float gscale, const float* stats, float* dz_low, float* workspace,
                    void* stream);

/* Fused capture + per-image aggregate: the capture branch (ptp_utils.py:508-538) of L
 * layers followed by collect_maps' mean over layers and heads (optimize.py:27-79), per image,
 * with no (B·H, R², N) attention in memory:
 *   maps[b, n, p] = (1/(L·H)) Σ_l Σ_h softmax_n(bicubic_{s_l->R}(z_l[b·H + h, :, n])[p]).
 * z_low: host array of L device pointers, layer l (B·H, s_l², N), 16-B aligned when N % 4 == 0;
 * sizes: host array of the L s_l (1 <= s_l <= R); maps (B, N, R*R).
 * stats: NULL or a host array of L device pointers (entries may be NULL), layer l
 * (B·H, R*R, 2) receiving each pixel's softmax (max, 1/Σexp) exactly as skp_capture_fwd's
 * `stats`, for skp_capture_bwd.                                                   */
int skp_capture_maps_fwd(const float* const* z_low, const int* sizes, int L, int B, int H, int N, int R, float* maps,
                         float* const* stats, void* stream);

/* Backward of skp_capture_maps_fwd for all L layers: dz_low[l] = bicubicᵀ(a ⊙ (g − Σ_n a g))
 * per (b·H + h) with g = gscale · dmaps[b] (the per-image map gradient broadcast over heads,
 * gscale = 1/(L·H) for the mean) and a rebuilt from the forward's stats (NULL: recomputed).
 * dmaps (B, N, R*R) token-major; dz_low: host array of L device pointers, (B·H, s_l², N).
 * N % 4 == 0.  workspace: B·R²·N + B·H·R·max(s_l)·N floats, 16-B aligned (pixel-major gradient
 * copy + row partials).  Deterministic (no atomics).                                   */
int skp_capture_maps_bwd(const float* const* z_low, const int* sizes, int L, int B, int H, int N, int R,
                         const float* dmaps, float gscale, const float* const* stats, float* const* dz_low,
                         float* workspace, void* stream);

/* Backward of skp_capture_maps_fwd for a SPARSE per-image map gradient — the token-opt losses
 * read only the selected token rows maps[b, tok] (optimize.py:403-424 sharpening / equivariance
 * on top_embedding_indices), so image b's gradient is gsel[b, k] (R*R) at token sel_tok[b, k]
 * (int64, −1 = unused slot; duplicates add), zero elsewhere.  Same result as
 * skp_capture_maps_bwd on the scattered dense gradient, without forming it:
 *   dZ = a ⊙ (g − dot) = [a_k·g_k at the K selected tokens] − dot·a,  dot = Σ_k a_k·g_k,
 * the dense part needing one scalar per pixel.  K <= 32, N % 4 == 0, stats REQUIRED (the
 * forward's), dz_low / z_low 16-B aligned.  workspace: skp_capture_maps_bwd_sel_workspace()
 * floats, 16-B aligned (returns -1 on a bad shape).  R = s·{4, 8, 16} for R in {32, 64, 128}
 * take the fast kernels; other shapes scatter into a dense gradient and run
 * skp_capture_maps_bwd.  Deterministic (no atomics).                                   */
long long skp_capture_maps_bwd_sel_workspace(const int* sizes, int L, int B, int H, int N, int R, int K);
int skp_capture_maps_bwd_sel(const float* const* z_low, const int* sizes, int L, int B, int H, int N, int R,
                             const long long* sel_tok, int K, const float* gsel, float gscale,
                             const float* const* stats, float* const* dz_low, float* workspace, void* stream);
/* Per-phase device time of skp_capture_maps_bwd_sel's fast path (measurement only, not on the
 * reference's interface): skp_sel_bwd_timing(1) makes every later single-stream call record HIP
 * events between its phases on its stream (at most 256 calls), skp_sel_bwd_timing(0) stops;
 * skp_sel_bwd_timing_read waits for the recorded calls and returns the summed ms of
 * ms[0] sel_gather, ms[1] sel_doth (sel_dot), ms[2] the adjoint's vertical pass (sel_adjw), ms[3]
 * sel_dense, and the number of calls, then clears the record.                              */
int skp_sel_bwd_timing(int enable);
int skp_sel_bwd_timing_read(double* ms, int* calls);

/* ---------------------------------------------------------------- A3 aggregate
 * optimize.collect_maps (optimize.py:27-79), token-major output:
 * out[m, p] = (1/(L·BH)) Σ_l Σ_b attn_l[b, p, idx(m)], idx = indices[m] or m.
 * layers: host array of L device pointers, each (BH, RR, N).                  */
int skp_aggregate(const float* const* layers, int L, int BH, int RR, int N, const long long* indices,
                  int n_out, float* out, void* stream);

/* Bilinear resize (F.interpolate mode="bilinear", align_corners=False; optimize.py:63-70)
 * of C square planes R×R -> Ro×Ro, and its adjoint.                            */
int skp_resize_bilinear(const float* in, int C, int R, int Ro, float* out, void* stream);
int skp_resize_bilinear_bwd(const float* gout, int C, int R, int Ro, float* gin, void* stream);

/* ---------------------------------------------------------------- A4-A6 argmax family
 * eval.find_max_pixel (eval.py:39-60): first-occurrence argmax, NaN is max.
 * rows: optional device list of n_rows row ids (NULL = rows 0..T-1).
 * pos (n_rows, 2) = (idx / w + 0.5, idx % w + 0.5); idx (n_rows) optional.     */
int skp_argmax2d(const float* maps, int T, int h, int w, const long long* rows, int n_rows, float* pos,
                 long long* idx, void* stream);

/* eval.find_k_max_pixels + mask_radius (eval.py:62-111): `num` rounds of argmax,
 * each followed by map *= (squared distance > radius2).  pos (num, T, 2).
 * masked (T, h, w) optional: the map after the last round's mask.             */
int skp_k_max_pixels(const float* maps, int T, int h, int w, int num, float radius2, float* pos,
                     float* masked, void* stream);

/* eval.mask_radius (eval.py:83-111): out = map * (squared distance to pos > radius2). */
int skp_mask_radius(const float* maps, int T, int h, int w, const float* pos, float radius2, float* out,
                    void* stream);

/* eval.pixel_from_weighted_avg (eval.py:113-155): zero pixels farther than
 * `distance` from the argmax (in place when mutate != 0, like the reference),
 * then the normalised centroid + 0.5.  distance < 0 disables the cut.          */
int skp_weighted_avg(float* maps, int T, int h, int w, float distance, int mutate, float* pos, void* stream);

/* ---------------------------------------------------------------- A7 target
 * optimize_token.gaussian_circles (optimize_token.py:204-242):
 * out[t,i,j] = mean_q exp(-((j+.5-P[q,t,1]·size)² + (i+.5-P[q,t,0]·size)²)/(2σ²)),
 * P = pos (num, T, 2) in [0, 1].                                               */
int skp_gaussian_target(const float* pos, int num, int T, int size, float sigma, float* out, void* stream);

/* ---------------------------------------------------------------- A8-A10 select
 * ptp_utils.find_top_k_gaussian (ptp_utils.py:86-112): per-token
 * KL(normalised G(argmax)+eps ‖ softmax(map+eps)), ascending, first top_k
 * (ties by token id).  kl (T) doubles optional; workspace >= 16*T bytes.       */
int skp_topk_gaussian(const float* maps, int T, int h, int w, int top_k, float sigma, float epsilon,
                      int num_subjects, long long* out, double* kl, void* workspace, void* stream);

/* skp_topk_gaussian for nb images in one launch (each image's top-k chosen as the reference's
 * find_top_k_gaussian on that image, ptp_utils.py:86-112; optimize.py:403-410 per replica):
 * maps (nb, T, h, w), out (nb, top_k), kl (nb, T) optional, workspace >= 16*nb*T bytes.      */
int skp_topk_gaussian_batch(const float* maps, int nb, int T, int h, int w, int top_k, float sigma,
                            float epsilon, int num_subjects, long long* out, double* kl, void* workspace,
                            void* stream);

/* The ranking step of find_top_k_gaussian / entropy_sort (`torch.argsort(keys)[:top_k]`,
 * ptp_utils.py:110-112 and :185) for nb segments of T fp64 keys: ascending, NaN last, ties by
 * index; keys (nb, T), out (nb, top_k).  skp_topk_gaussian_batch with top_k = 0 and this call
 * together are skp_topk_gaussian_batch with top_k > 0.                                        */
int skp_topk_keys(const double* keys, int nb, int T, int top_k, long long* out, void* stream);

/* ptp_utils.entropy_sort (ptp_utils.py:165-187): ascending softmax entropy.     */
int skp_entropy_sort(const float* maps, int T, int h, int w, int top_k, long long* out, double* ent,
                     void* workspace, void* stream);

/* ptp_utils.furthest_point_sampling (ptp_utils.py:115-159) on the argmax positions
 * of the candidate rows; strict '>' first-wins, IEEE sqrt distances.
 * out[top_k] (int64); n_out (device int) = how many were selected.
 * workspace >= 16 * n_cand bytes.                                              */
int skp_fps(const float* maps, int T, int h, int w, const long long* cand, int n_cand, int top_k,
            long long* out, int* n_out, void* workspace, void* stream);
/* skp_fps for nb images in one launch (ptp_utils.py:115-159 per replica, optimize.py:419-424):
 * maps (nb, T, h, w), cand (nb, n_cand) token ids of each image, out (nb, top_k), n_out (nb),
 * workspace >= 8 * nb * n_cand bytes.                                                        */
int skp_fps_batch(const float* maps, int nb, int T, int h, int w, const long long* cand, int n_cand, int top_k,
                  long long* out, int* n_out, void* workspace, void* stream);
/* The ranking of skp_topk_keys and the candidates' argmax of skp_fps_batch in one launch, then the
   FPS launch: per image b, cand[b] = the n_cand tokens of smallest keys[b] (ascending; NaN last,
   ties by index — torch.argsort(keys)[:n_cand] of find_top_k_gaussian, ptp_utils.py:110-112), and
   out[b] / n_out[b] = furthest_point_sampling(maps[b], top_k, cand[b]) (ptp_utils.py:115-159) on the
   (nb, T, h, w) maps the FPS reads (the warped image's, optimize.py:403-410).  workspace: 2·nb·n_cand
   floats. */
int skp_fps_keys_batch(const double* keys, const float* maps, int nb, int T, int h, int w, int n_cand, int top_k,
                       long long* cand, long long* out, int* n_out, void* workspace, void* stream);

/* ---------------------------------------------------------------- A11 sharpening
 * optimize.sharpening_loss (optimize.py:166-206): pos = k-max of A / w,
 * G = gaussian_circles(pos, h, σ), loss = mean((A-G)²).
 * pos (num, T, 2) is written for the backward; partial >= T doubles.          */
int skp_sharpen_fwd(const float* A, int T, int h, int w, float sigma, int num_subjects, float* pos,
                     double* partial, float* loss, void* stream);
/* dA = gout[0] · 2(A − G)/numel.                                               */
int skp_sharpen_bwd(const float* A, int T, int h, int w, float sigma, int num_subjects, const float* pos,
                     const float* gout, float* dA, void* stream);
/* The sharpening loss of nb images at once (optimize.py:425-437 per replica): A (nb, T, h, w),
 * loss (nb) = each image's mean, pos (num, nb·T, 2), partial >= nb·T doubles; backward with
 * gout (nb).  Each image's loss and gradient are the single-image call's, bit for bit.        */
int skp_sharpen_fwd_batch(const float* A, int nb, int T, int h, int w, float sigma, int num_subjects, float* pos,
                          double* partial, float* loss, void* stream);
int skp_sharpen_bwd_batch(const float* A, int nb, int T, int h, int w, float sigma, int num_subjects,
                          const float* pos, const float* gout, float* dA, void* stream);

/* ---------------------------------------------------------------- A12 warp / equivariance
 * F.grid_sample(x, F.affine_grid(theta), bilinear, zeros, align_corners=False)
 * (invertable_transform.py:64-70, 86-90).  x (B, C, H, W), theta (B, 2, 3) device. */
int skp_affine_warp(const float* x, int B, int C, int H, int W, const float* theta, float* out, void* stream);
/* Adjoint w.r.t. x; gin is OVERWRITTEN (zeroed then accumulated).               */
int skp_affine_warp_bwd(const float* gout, int B, int C, int H, int W, const float* theta, float* gin,
                        void* stream);

/* optimize.equivariance_loss (optimize.py:157-163) for one replica:
 * loss = mean((A − warp(At, theta_inv))²), theta_inv (2,3) the inverse of that
 * replica's theta (invertable_transform.py:72-92).  partial >= T doubles.        */
int skp_equiv_fwd(const float* A, const float* At, int T, int h, int w, const float* theta_inv,
                  double* partial, float* loss, void* stream);
/* dA = gout·2(A−A')/numel (optional), dAt = warpᵀ(−dA) (overwritten).          */
int skp_equiv_bwd(const float* A, const float* At, int T, int h, int w, const float* theta_inv,
                  const float* gout, float* dA, float* dAt, void* stream);
/* The equivariance loss of nb replicas at once: A, At (nb, T, h, w), theta_inv (nb, 2, 3),
 * loss (nb), partial >= nb·T doubles; backward with gout (nb).  Same per-image values.       */
int skp_equiv_fwd_batch(const float* A, const float* At, int nb, int T, int h, int w, const float* theta_inv,
                        double* partial, float* loss, void* stream);
int skp_equiv_bwd_batch(const float* A, const float* At, int nb, int T, int h, int w, const float* theta_inv,
                        const float* gout, float* dA, float* dAt, void* stream);

/* ---------------------------------------------------------------- Winograd as batched GEMMs
 * The frozen UNet's small-image 3×3 convolutions (SD-1.5 ResnetBlock2D conv1/conv2 at 8²-32²):
 * F(4×4, 3×3) with the fused kernels' points, as V = Bᵀ d B → M[p] = V[p]ᵀ U[p] (36 batched
 * library GEMMs, host side) → y = Aᵀ M A (+ bias[k]) (+ residual).
 * V (36, C, T) and M (36, T, K), T = B·(H/4)·(W/4) tiles, t = (b·H/4 + ty)·W/4 + tx.          */
int skp_wino_in_transform(const float* x, int B, int C, int H, int W, float* V, void* stream);
int skp_wino_out_transform(const float* M, int B, int K, int H, int W, const float* bias, const float* residual,
                           float* y, void* stream);
/* skp_wino_out_transform with the GEMM product laid out M[p][k][t] (the operands swapped: M[p] =
 * U[p]ᵀ · V[p]), so the tiles leave as coalesced image-row runs; gn_part (optional): the next
 * GroupNorm's (mean, M2) per (image, channel, segment of min(P, 64) tiles), P = (H/4)·(W/4) tiles per
 * plane (16, 32 or a multiple of 64), nseg = P / min(P, 64) — the layout skp_groupnorm_fwd_part
 * reads. */
int skp_wino_out_transform_kt(const float* M, int B, int K, int H, int W, const float* bias, const float* residual,
                              float* y, float* gn_part, void* stream);

/* ---------------------------------------------------------------- Q·Kᵀ (fp32 MFMA)
 * C[b,m,n] = alpha · Σ_k A[b,m,k] · B[b,k,n] (+ C if accumulate), arbitrary element
 * strides; exact-f32 v_mfma_f32_32x32x2_f32.  Used for the capture logits
 * z = q kᵀ·scale (ptp_utils.py:493/534) and their gradients.                   */
int skp_bgemm_f32(const float* A, long long sAb, long long sAm, long long sAk, const float* B, long long sBb,
                  long long sBk, long long sBn, float* C, long long sCb, long long sCm, long long sCn, int batch,
                  int M, int N, int K, float alpha, int accumulate, void* stream);
/* skp_bgemm_f32 with a two-level batch: batch index z = o·hb + i, operand X's base X + o·sXo + i·sXb.
 * Reads attention heads in place from the (B, S, H·d) projections (sXo = S·H·d, sXb = d, row stride
 * H·d) and an operand shared by the B images with sXo = 0 — the captured layers' q·kᵀ and P·v with
 * the batch-shared token embedding (ptp_utils.py:481-536) without head-permute or batch-expand copies.
 * skp_bgemm_f32 is the hb = batch, sXo = 0 case. */
int skp_bgemm_f32_2b(const float* A, long long sAo, long long sAb, long long sAm, long long sAk, const float* B,
                     long long sBo, long long sBb, long long sBk, long long sBn, float* C, long long sCo, long long sCb,
                     long long sCm, long long sCn, int batch, int hb, int M, int N, int K, float alpha, int accumulate,
                     void* stream);

/* ---------------------------------------------------------------- UNet-side: GroupNorm (+SiLU)
 * The token-opt backward runs through the frozen SD-1.5 UNet; its
 * GroupNorm → SiLU pairs (diffusers-0.8.0 ResnetBlock2D / Transformer2DModel.norm /
 * VAE encoder) run fused here.  x, y, dx: (B, C, HW) NCHW fp32; act = 1 applies SiLU.
 * shift (B*C floats, or NULL) is added to x on load: GroupNorm(x + shift[b, c]) — the
 * preceding convolution's bias and the resnet's time embedding, never materialised.
 * stats (B*G*2 floats) = (mean, rstd) per group, written by fwd and read by bwd.
 * partial: skp_groupnorm_workspace(B, C, HW, G) doubles.  Parameters are frozen, so the
 * backward returns dx only.                                                      */
int skp_groupnorm_workspace(int B, int C, long long HW, int G);
int skp_groupnorm_fwd(const float* x, const float* gamma, const float* beta, const float* shift, int B, int C,
                      long long HW, int G, float eps, int act, float* y, float* stats, double* partial,
                      void* stream);
int skp_groupnorm_bwd(const float* x, const float* dy, const float* gamma, const float* beta, const float* shift,
                      const float* stats, int B, int C, long long HW, int G, int act, float* dx, double* partial,
                      void* stream);
/* skp_groupnorm_fwd with the statistics pass replaced by the producing convolution's per-segment
 * statistics: part (B, C, nseg) float2 (mean, M2 = Σ(x − mean)²) per segment of n = HW / nseg
 * pixels, as skp_conv3x3_wino2_gn / skp_wino_out_transform_kt write them; combined in fp64 by
 * Chan's formula with the shift folded into each segment mean.  Same output and saved
 * (mean, rstd) layout. */
int skp_groupnorm_fwd_part(const float* x, const float* gamma, const float* beta, const float* shift, const float* part,
                           int nseg, int B, int C, long long HW, int G, float eps, int act, float* y, float* stats,
                           double* partial, void* stream);
/* skp_groupnorm_bwd plus dres (may be null): dx = GroupNorm-backward(dy) + dres, the gradient of x's
 * other consumer (the ResNet block's residual or shortcut, the spatial transformer's residual) added
 * in the same pass instead of by the autograd engine (diffusers resnet.py / attention.py residuals). */
int skp_groupnorm_bwd_add(const float* x, const float* dy, const float* gamma, const float* beta, const float* shift,
                          const float* stats, int B, int C, long long HW, int G, int act, const float* dres, float* dx,
                          double* partial, void* stream);
/* Softmax backward of the UNet's math attention (diffusers-0.8.0 CrossAttention,
 * softmax(q kᵀ·scale) v): per row of P (rows × cols), dS = alpha·P ⊙ (dP − Σ P ⊙ dP),
 * written over dP (alpha = the logits' scale, baddbmm's backward folded in).  cols ≤ 16384. */
int skp_softmax_bwd(const float* P, float* dP, long long rows, int cols, float alpha, void* stream);
/* Its forward, in place: S (rows × cols, cols % 4 == 0, ≤ 16384) ← softmax over each row
 * (torch order: max-subtracted exp, divided by the row sum).  One read and one write of S
 * (the (B·H, 4096, 4096) scores of the 64²-token layers are 4.3 GB at batch 8).           */
int skp_softmax_fwd(float* S, long long rows, int cols, void* stream);
/* Fused score gradient of the math attention's backward: out = alpha·P ⊙ (dO·Vᵀ − D) with
 * dO·Vᵀ on the f32 matrix cores (never materialised) and D[row] = dO_row·O_row (the forward
 * output); P (BH, S, L), dO (BH, S, d), V (BH, L, d), D (BH, S).  out may alias P.
 * S, L multiples of 64; d ∈ {40, 64, 80, 160}.                                         */
int skp_attn_dscore(const float* P, const float* dO, const float* V, const float* D, float* out, int BH, int S, int L,
                    int d, float alpha, void* stream);
/* Fused attention backward over key blocks: dS = alpha·P⊙(dO·Vᵀ − D) written to dS (as
 * skp_attn_dscore) and, from the same registers, dV = Pᵀ·dO and dK = dSᵀ·Q (so dK carries
 * alpha).  P, dS (BH, S, L); dO, Q (BH, S, d); V, dV, dK (BH, L, d); D = rowsum(dO⊙O) (BH, S).
 * S, L multiples of 64; d ∈ {40, 64, 80}; dO, Q, V, dV, dK 16-byte aligned.  Replaces the
 * autograd backward of diffusers' CrossAttention baddbmm → softmax → bmm (attention.py).     */
int skp_attn_bwd_kv(const float* P, const float* dO, const float* Q, const float* V, const float* D, float* dS,
                    float* dV, float* dK, int BH, int S, int L, int d, float alpha, void* stream);
/* Fused attention O = softmax(scale·Q Kᵀ) V (online softmax; no score tensor); with stats
 * non-null also the per-row (max, 1/sum) pairs (BH, S, 2) that skp_attn_bwd_flash consumes.
 * Q (BH, S, d), K, V (BH, L, d), O (BH, S, d); S a multiple of 64, L any (the last key block
 * is masked); d ∈ {40, 64, 80}.                                                  */
int skp_attn_fwd(const float* Q, const float* K, const float* V, float* O, float* stats, int BH, int S, int L, int d,
                 float scale, void* stream);
/* Attention backward that rebuilds P = exp(scale·Q Kᵀ − m) · (1/l) per key block from the
 * forward's row stats (stats from skp_attn_fwd, (BH, S) × (m, 1/l)) instead of reading a saved P:
 * dS (BH, S, L) = scale·P⊙(dO·Vᵀ − D), dV = Pᵀ·dO, dK = dSᵀ·Q; dQ = dS·K is left to a GEMM.
 * Q, dO (BH, S, d); K, V, dV, dK (BH, L, d); D = rowsum(dO⊙O) (BH, S).  S a multiple of 64,
 * L any; d ∈ {40, 64, 80}; 16-byte aligned (stats 8).                                                  */
int skp_attn_bwd_flash(const float* Q, const float* K, const float* V, const float* dO, const float* stats,
                       const float* D, float* dS, float* dV, float* dK, int BH, int S, int L, int d, float scale,
                       void* stream);
/* skp_attn_fwd / skp_attn_bwd_flash on the projections' own layout, without the head permutes of
 * diffusers' reshape_heads_to_batch_dim / reshape_batch_dim_to_heads (CrossAttention.forward,
 * reference ptp_utils.py:481-506 for the layers the capture does not patch): element (b, h, s, j)
 * of Q / K / V / O / dO / dV / dK sits at base + b·sb + s·rs + h·d + j (a (B, S, H·d) tensor:
 * sb = S·H·d, rs = H·d; a context shared by the batch: sb = 0 — then dK / dV still get their own
 * per-image rows and the caller sums them).  stats (B·H, S, 2), D (B·H, S), dS (B·H, S, L)
 * contiguous, as in the (B·H, S, d) entries; strides multiples of 4, 16-byte aligned.         */
int skp_attn_fwd_bshd(const float* Q, long long q_sb, int q_rs, const float* K, long long k_sb, int k_rs,
                      const float* V, long long v_sb, int v_rs, float* O, long long o_sb, int o_rs, float* stats, int B,
                      int H, int S, int L, int d, float scale, void* stream);
int skp_attn_bwd_flash_bshd(const float* Q, long long q_sb, int q_rs, const float* K, long long k_sb, int k_rs,
                            const float* V, long long v_sb, int v_rs, const float* dO, long long o_sb, int o_rs,
                            const float* stats, const float* D, float* dS, float* dV, long long dv_sb, int dv_rs,
                            float* dK, long long dk_sb, int dk_rs, int B, int H, int S, int L, int d, float scale,
                            void* stream);
/* LayerNorm over the last dimension (the UNet transformer blocks' norm1/2/3; frozen γ, β):
 * x, y (rows, C), C a multiple of 4 ≤ 2048; stats (rows, 2) = (mean, 1/sqrt(var + eps)) for the
 * backward, which gives dx = rstd·(dy·γ − mean(dy·γ) − x̂·mean(dy·γ·x̂)).  Replaces
 * torch.nn.LayerNorm inside diffusers' BasicTransformerBlock (attention.py).               */
int skp_layernorm_fwd(const float* x, const float* gamma, const float* beta, long long rows, int C, float eps, float* y,
                      float* stats, void* stream);
int skp_layernorm_bwd(const float* x, const float* dy, const float* gamma, const float* stats, long long rows, int C,
                      float* dx, void* stream);
/* skp_layernorm_bwd plus dres (may be null): dx = LayerNorm-backward(dy) + dres, the transformer
 * block's residual gradient (h = attn(norm(h)) + h, diffusers attention.py) added in the same pass. */
int skp_layernorm_bwd_add(const float* x, const float* dy, const float* gamma, const float* stats, long long rows,
                          int C, const float* dres, float* dx, void* stream);
/* diffusers GEGLU (the UNet FeedForward's proj → chunk(2) → x·gelu(gate), exact-erf GELU):
 * h (rows, 2I) → out (rows, I), and its backward dh (rows, 2I) from dout (rows, I).
 * I % 4 == 0, 16-byte aligned.                                                 */
int skp_geglu_fwd(const float* h, long long rows, int I, float* out, void* stream);
int skp_geglu_bwd(const float* h, const float* dout, long long rows, int I, float* dh, void* stream);
/* out = a + (h + bias[c]) over (B, C, HW): diffusers ResnetBlock2D `x + conv2(...)` with the
 * convolution's bias folded into the residual add (same rounding order).         */
int skp_residual_bias_add(const float* a, const float* h, const float* bias, int B, int C, long long HW,
                          float* out, void* stream);
/* 3×3 / stride-1 / pad-1 convolution of the frozen VAE encoder and UNet (diffusers Conv2d in
 * Encoder / ResnetBlock2D / Upsample2D, run by ptp_utils.py:289-304 image2latent and the UNet
 * forward/backward of optimize.py:173-190) as Winograd F(4×4, 3×3) on the fp32 matrix cores.
 * skp_wino_weights: transformed weights U (K·C·36 floats, layout [K/32][C][32][36]) from
 *   w (K, C, 3, 3) (flip 0), or, for the input gradient, from the forward weight w (C, K, 3, 3)
 *   rotated 180° and transposed (flip 1).  K % 32 == 0.
 * skp_conv3x3_wino: y (B, K, H, W) = conv(x (B, C, H, W), w) + bias[k] (bias may be NULL)
 *   + residual (B, K, H, W) (may be NULL).  C % 4 == 0, K % 32 == 0, H % 4 == W % 4 == 0,
 *   16-byte aligned tensors.  nsplit > 1 splits the input channels over nsplit workgroup sets
 *   (C % (4·nsplit) == 0) for grids too small to fill the chip: partial sums go to ws
 *   (nsplit·B·K·H·W floats) and one pass adds them (in split order), the bias and the
 *   residual into y.  nsplit == 1: ws unused (may be NULL).                     */
int skp_wino_weights(const float* w, int K, int C, int flip, float* U, void* stream);
int skp_conv3x3_wino(const float* x, const float* U, const float* bias, const float* residual, float* y, int B, int C,
                     int K, int H, int W, int nsplit, float* ws, void* stream);
/* The same convolution for H % 32 == W % 32 == 0 (workgroup = 32×32 output pixels × 32
 * channels, three stages of input region and weights in flight, transforms straight into the
 * MFMA operands).  skp_wino2_weights writes U as [K/32][C][32][40] (positions 0..17 at 0..17,
 * 18..35 at 20..37, zero pads); flip as above.  Also 16×16 images with B % 4 == 0 (four
 * whole images per workgroup).  */
int skp_wino2_weights(const float* w, int K, int C, int flip, float* U, void* stream);
int skp_conv3x3_wino2(const float* x, const float* U, const float* bias, const float* residual, float* y, int B,
                      int C, int K, int H, int W, int nsplit, float* ws, void* stream);
/* skp_conv3x3_wino2 that also writes the next GroupNorm's statistics from its epilogue: gn_part
 * (B, K, H/16 · W/32) float2 = (mean, M2 = Σ(y − mean)²) of the final output (bias and residual
 * included) per channel over each 16-row × 32-pixel segment, accumulated around a pivot value of
 * the segment (nsplit = 1, H and W multiples of 32; may be null).  The
 * consumer is skp_groupnorm_fwd_part: the frozen UNet / VAE's GroupNorm(+SiLU) after a 3×3 convolution
 * (diffusers resnet.py) then reads its input once instead of twice. */
int skp_conv3x3_wino2_gn(const float* x, const float* U, const float* bias, const float* residual, float* y, int B,
                         int C, int K, int H, int W, int nsplit, float* ws, float* gn_part, void* stream);
/* diffusers' Downsample2D(padding=0) of the VAE encoder (F.pad(x, (0, 1, 0, 1)) then a 3×3 stride-2
 * convolution; the encoder behind ptp_utils.image2latent, reference ptp_utils.py:289-304):
 * y (B, K, H/2, W/2) = the stride-1 pad-1 convolution of x sampled at (2oy + 1, 2ox + 1), + bias,
 * computed by the skp_conv3x3_wino2 kernel (U from skp_wino2_weights) with a stride-2 epilogue.
 * H, W multiples of 32; C % 4 == 0, K % 32 == 0; nsplit as skp_conv3x3_wino2 (workspace
 * nsplit·B·K·(H/2)·(W/2) floats).                                                              */
int skp_conv3x3s2_wino2(const float* x, const float* U, const float* bias, float* y, int B, int C, int K, int H,
                        int W, int nsplit, float* ws, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SKP_H */
