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
