// Winograd F(4×4, 3×3) as transform → 36 batched GEMMs → inverse transform, for the frozen
// UNet's small-image, many-channel 3×3 convolutions (8², 16², 32²; reference: the SD-1.5
// ResnetBlock2D conv1 / conv2 the token-optimisation backward runs through).
//
// The fused kernels (skp_conv.hip) transform, multiply and inverse-transform inside one
// workgroup; at these sizes a convolution has few tiles per channel, so their grids are a few
// hundred workgroups whose per-stage latency, not the matrix cores, sets the time (the 16² ×
// 1280 → 1280 layer at 38% MFMA-busy).  Here the two transforms are bandwidth-light VALU passes
// and the multiply is one batched library GEMM per convolution (36 positions × (tiles × C) ·
// (C × K)), which runs near the f32 matrix-core rate:
//   skp_wino_in_transform   x (B, C, H, W) → V[p][c][t] = (Bᵀ d_t,c B)[p]
//   (GEMM, host side)       M[p] = V[p]ᵀ · U[p]            (T × K per position)
//   skp_wino_out_transform  M[p][t][k] → y[b][k][4ty + r][4tx + s] = (Aᵀ M A)[r][s] (+ bias, + res)
// t = (b·(H/4) + ty)·(W/4) + tx.  The points (0, 1, −1, 1/2, −2, ∞) and the matrices are the
// fused kernels' (skp_conv.hip kBt / kAt / Gm), so both forms compute the same transform.
#include "skp_common.h"

using namespace skp;

namespace {

// Bᵀ (rows i = transform row, columns a = patch row) and Aᵀ for the points (0, 1, −1, 1/2, −2, ∞)
__device__ constexpr float kBt[6][6] = {{1.f, -1.5f, -2.f, 1.5f, 1.f, 0.f},  {0.f, -1.f, 0.5f, 2.5f, 1.f, 0.f},
                                        {0.f, 1.f, -2.5f, 0.5f, 1.f, 0.f},  {0.f, -2.f, -1.f, 2.f, 1.f, 0.f},
                                        {0.f, 0.5f, -1.f, -0.5f, 1.f, 0.f}, {0.f, 1.f, -1.5f, -2.f, 1.5f, 1.f}};
__device__ constexpr float kAt[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                                        {0.f, 1.f, -1.f, 0.5f, -2.f, 0.f},
                                        {0.f, 1.f, 1.f, 0.25f, 4.f, 0.f},
                                        {0.f, 1.f, -1.f, 0.125f, -8.f, 1.f}};

// one thread per (channel, tile); a block's threads take consecutive tiles of one channel, so the
// 36 stores per thread are coalesced runs over t and the patch loads overlap between neighbours
// (a flattened channel-major grid that keeps blocks full below 256 tiles per channel measured
// 13.7 vs 12.9 µs per launch in the bench, r05x vs r05p traces, and was not kept)
__global__ __launch_bounds__(256) void wino_in_kernel(const float* __restrict__ x, int B, int C, int H, int W,
                                                      float* __restrict__ V) {
  const int tw = W >> 2, th = H >> 2, T = B * th * tw;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (t >= T) return;
  const int b = t / (th * tw), r = t - b * th * tw;
  const int ty = r / tw, tx = r - ty * tw;
  const float* xc = x + ((size_t)b * C + c) * H * W;
  float d[6][6];
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    const int yy = 4 * ty - 1 + a;
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const int xx = 4 * tx - 1 + e;
      d[a][e] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? xc[(size_t)yy * W + xx] : 0.0f;
    }
  }
  float tmp[6][6];   // tmp = Bᵀ d
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      float s = 0.0f;
#pragma unroll
      for (int a = 0; a < 6; ++a)
        if (kBt[i][a] != 0.0f) s = fmaf(kBt[i][a], d[a][e], s);
      tmp[i][e] = s;
    }
  const size_t ps = (size_t)C * T;
  float* out = V + (size_t)c * T + t;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {   // (Bᵀ d B)[i][j] = Σ_e tmp[i][e] Bᵀ[j][e]
      float s = 0.0f;
#pragma unroll
      for (int e = 0; e < 6; ++e)
        if (kBt[j][e] != 0.0f) s = fmaf(tmp[i][e], kBt[j][e], s);
      out[(size_t)(6 * i + j) * ps] = s;
    }
}

// one thread per (tile, output channel): the 36 loads per thread are coalesced over k; the 4×4
// output tile leaves as four 16-B row stores (+ bias, + residual: (acc + bias) + res)
__global__ __launch_bounds__(256) void wino_out_kernel(const float* __restrict__ M, int B, int K, int H, int W,
                                                       const float* __restrict__ bias, const float* __restrict__ res,
                                                       float* __restrict__ y) {
  const int tw = W >> 2, th = H >> 2, T = B * th * tw;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = blockIdx.y;
  if (k >= K) return;
  const int b = t / (th * tw), r = t - b * th * tw;
  const int ty = r / tw, tx = r - ty * tw;
  const size_t ps = (size_t)T * K;
  const float* m = M + (size_t)t * K + k;
  float mv[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) mv[i][j] = m[(size_t)(6 * i + j) * ps];
  float tmp[4][6];   // Aᵀ M
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int i = 0; i < 6; ++i)
        if (kAt[q][i] != 0.0f) s = fmaf(kAt[q][i], mv[i][j], s);
      tmp[q][j] = s;
    }
  const float bk = bias ? bias[k] : 0.0f;
  const size_t base = ((size_t)b * K + k) * H * W + (size_t)(4 * ty) * W + 4 * tx;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float o[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      float s = 0.0f;
#pragma unroll
      for (int j = 0; j < 6; ++j)
        if (kAt[s2][j] != 0.0f) s = fmaf(tmp[q][j], kAt[s2][j], s);
      o[s2] = s;
    }
    const size_t off = base + (size_t)q * W;
    float4 v = make_float4(o[0], o[1], o[2], o[3]);
    if (bias) {
      v.x += bk; v.y += bk; v.z += bk; v.w += bk;
    }
    if (res) {
      const float4 rv = *reinterpret_cast<const float4*>(res + off);
      v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
    }
    *reinterpret_cast<float4*>(y + off) = v;
  }
}

// The same inverse transform with the GEMM's product laid out [p][k][t] (M[p] = U[p]ᵀ · V[p], the
// operands swapped): one thread per (output channel, tile), a block's threads over consecutive
// tiles of one channel, so the 36 loads per thread are coalesced over t AND the 4×4 tiles leave as
// contiguous image-row runs (the [p][t][k] form above stores one 16-B piece per lane into 64
// different channel planes).  gnp (optional): the next GroupNorm's (mean, M2) of the output per
// segment of min(P, 64) tiles of one channel plane (P = tiles per plane, 16, 32 or a multiple of
// 64), nseg = P / min(P, 64) per plane: (Σd, Σd²) around a pivot (the segment's first value),
// reduced over the segment's lanes, then mean = pivot + Σd/n, M2 = Σd² − (Σd)²/n.
__global__ __launch_bounds__(256) void wino_out_kt_kernel(const float* __restrict__ M, int B, int K, int H, int W,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ res, float* __restrict__ y,
                                                          float2* __restrict__ gnp) {
  const int tw = W >> 2, th = H >> 2, P = th * tw, T = B * P;
  // flattened (k, t), k-major: full blocks below 256 tiles per channel; a GroupNorm segment (an
  // aligned run of min(P, 64) tiles of one plane) stays inside a wave since K·T, T and P are
  // multiples of it
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = e < (long long)K * T;
  const long long ee = live ? e : (long long)K * T - 1;
  const int k = (int)(ee / T);
  const int tt = (int)(ee - (long long)k * T);
  const int b = tt / P, r = tt - b * P;
  const int ty = r / tw, tx = r - ty * tw;
  const size_t ps = (size_t)K * T;
  const float* m = M + (size_t)k * T + tt;
  float mv[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) mv[i][j] = m[(size_t)(6 * i + j) * ps];
  float tmp[4][6];   // Aᵀ M
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int i = 0; i < 6; ++i)
        if (kAt[q][i] != 0.0f) s = fmaf(kAt[q][i], mv[i][j], s);
      tmp[q][j] = s;
    }
  const float bk = bias ? bias[k] : 0.0f;
  const size_t base = ((size_t)b * K + k) * H * W + (size_t)(4 * ty) * W + 4 * tx;
  const int seg = P < 64 ? P : 64;
  float s1 = 0.0f, s2 = 0.0f, piv = 0.0f;   // (Σd, Σd²) of d = v − piv, piv = the segment's first value
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float o[4];
#pragma unroll
    for (int s2i = 0; s2i < 4; ++s2i) {
      float s = 0.0f;
#pragma unroll
      for (int j = 0; j < 6; ++j)
        if (kAt[s2i][j] != 0.0f) s = fmaf(tmp[q][j], kAt[s2i][j], s);
      o[s2i] = s;
    }
    const size_t off = base + (size_t)q * W;
    float4 v = make_float4(o[0], o[1], o[2], o[3]);
    if (bias) {
      v.x += bk; v.y += bk; v.z += bk; v.w += bk;
    }
    if (res) {
      const float4 rv = *reinterpret_cast<const float4*>(res + off);
      v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
    }
    if (live) *reinterpret_cast<float4*>(y + off) = v;
    if (gnp) {
      if (q == 0) piv = __shfl(v.x, (int)(threadIdx.x & 63) & ~(seg - 1), 64);   // the segment's lane 0
      const float dx = v.x - piv, dy = v.y - piv, dz = v.z - piv, dw = v.w - piv;
      s1 += (dx + dy) + (dz + dw);
      s2 += (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
  }
  if (gnp) {   // uniform: the segment's lanes all take part (segments are whole planes' tiles: all
               // live or all past the last image)
    if (!live) s1 = s2 = 0.0f;
    // reduce over aligned groups of `seg` lanes (16, 32 or 64; lanes of a segment are one plane)
    s1 += dpp_read<0xB1>(s1); s2 += dpp_read<0xB1>(s2);
    s1 += dpp_read<0x4E>(s1); s2 += dpp_read<0x4E>(s2);
    s1 += dpp_read<0x141>(s1); s2 += dpp_read<0x141>(s2);
    s1 += dpp_read<0x140>(s1); s2 += dpp_read<0x140>(s2);
    if (seg >= 32) { s1 += __shfl_xor(s1, 16, 64); s2 += __shfl_xor(s2, 16, 64); }
    if (seg >= 64) { s1 += __shfl_xor(s1, 32, 64); s2 += __shfl_xor(s2, 32, 64); }
    if (live && (threadIdx.x & (seg - 1)) == 0) {   // (mean, M2) of the segment's 16·seg outputs
      const int nseg = P / seg;
      const float inv_n = 1.0f / (float)(16 * seg);
      gnp[((size_t)b * K + k) * nseg + r / seg] = make_float2(piv + s1 * inv_n, fmaxf(s2 - s1 * (s1 * inv_n), 0.0f));
    }
  }
}

}  // namespace

extern "C" int skp_wino_in_transform(const float* x, int B, int C, int H, int W, float* V, void* stream) {
  SKP_CHECK_ARG(x && V, "null pointer");
  SKP_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0, "non-positive shape");
  SKP_CHECK_ARG(H % 4 == 0 && W % 4 == 0, "H and W must be multiples of 4");
  SKP_CHECK_ARG(C <= 65535, "C > 65535");
  const long long T = (long long)B * (H / 4) * (W / 4);
  SKP_CHECK_ARG(T * C * 36 < (1LL << 40), "too large");
  hipLaunchKernelGGL(wino_in_kernel, dim3((unsigned)((T + 255) / 256), C), dim3(256), 0, as_stream(stream), x, B, C, H, W,
                     V);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_wino_out_transform(const float* M, int B, int K, int H, int W, const float* bias,
                                      const float* residual, float* y, void* stream) {
  SKP_CHECK_ARG(M && y, "null pointer");
  SKP_CHECK_ARG(B > 0 && K > 0 && H > 0 && W > 0, "non-positive shape");
  SKP_CHECK_ARG(H % 4 == 0 && W % 4 == 0, "H and W must be multiples of 4");
  SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
                    (!residual || (reinterpret_cast<uintptr_t>(residual) & 15) == 0),
                "y and residual must be 16-B aligned");
  const long long T = (long long)B * (H / 4) * (W / 4);
  SKP_CHECK_ARG(T <= 65535, "more than 65535 tiles (grid y)");
  hipLaunchKernelGGL(wino_out_kernel, dim3((K + 255) / 256, (unsigned)T), dim3(256), 0, as_stream(stream), M, B, K, H,
                     W, bias, residual, y);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_wino_out_transform_kt(const float* M, int B, int K, int H, int W, const float* bias,
                                         const float* residual, float* y, float* gn_part, void* stream) {
  SKP_CHECK_ARG(M && y, "null pointer");
  SKP_CHECK_ARG(B > 0 && K > 0 && H > 0 && W > 0, "non-positive shape");
  SKP_CHECK_ARG(H % 4 == 0 && W % 4 == 0, "H and W must be multiples of 4");
  SKP_CHECK_ARG(K <= 65535, "more than 65535 output channels (grid y)");
  SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
                    (!residual || (reinterpret_cast<uintptr_t>(residual) & 15) == 0),
                "y and residual must be 16-B aligned");
  const long long P = (long long)(H / 4) * (W / 4), T = B * P;
  SKP_CHECK_ARG(T < (1LL << 31), "too many tiles");
  SKP_CHECK_ARG(!gn_part || ((P == 16 || P == 32 || P % 64 == 0) && (reinterpret_cast<uintptr_t>(gn_part) & 7) == 0),
                "gn_part: tiles per plane must be 16, 32 or a multiple of 64; 8-B aligned");
  SKP_CHECK_ARG(T * K < (1LL << 40), "too large");
  hipLaunchKernelGGL(wino_out_kt_kernel, dim3((unsigned)((T * K + 255) / 256)), dim3(256), 0, as_stream(stream), M, B,
                     K, H, W, bias, residual, y, reinterpret_cast<float2*>(gn_part));
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
