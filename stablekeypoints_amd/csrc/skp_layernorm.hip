// LayerNorm over the last dimension (the UNet transformer blocks' norm1/2/3, frozen affine
// parameters, input gradient only) on gfx950.  The rows are short (C = 320 / 640 / 1280 in
// SD-1.5), so one wave owns a row and keeps it in registers (float4 per lane) between the
// mean, the variance and the normalisation: one read and one write of x per pass, where
// ATen's kernel runs at ≈1.7 TB/s on these shapes.
//   forward:  mean, rstd = 1/sqrt(var + eps) (biased variance, two-pass), y = x̂·γ + β;
//             (mean, rstd) per row saved for the backward
//   backward: g = dy·γ, dx = rstd·(g − mean(g) − x̂·mean(g·x̂)) [+ dres: the gradient of the other
//             consumer of x — the transformer block's residual — added in the same pass]
#include "skp_common.h"

using namespace skp;

namespace {

constexpr int kRowsPerBlock = 4;   // one wave per row

template <int NQ>   // float4 per lane: C / 4 <= 64·NQ
__global__ __launch_bounds__(64 * kRowsPerBlock) void ln_fwd_kernel(const float* __restrict__ x,
                                                                    const float* __restrict__ gamma,
                                                                    const float* __restrict__ beta, long long rows,
                                                                    int C, float eps, float* __restrict__ y,
                                                                    float2* __restrict__ stats) {
  const long long row = (long long)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63, C4 = C >> 2;
  const float4* xr = reinterpret_cast<const float4*>(x + row * C);
  float4 v[NQ];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = lane + 64 * i;
    v[i] = q < C4 ? xr[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.0f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    if (lane + 64 * i < C4) {
      const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
      ss += (a * a + b * b) + (c * c + d * d);
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)C + eps);
  float4* yr = reinterpret_cast<float4*>(y + row * C);
  const float4* g4 = reinterpret_cast<const float4*>(gamma);
  const float4* b4 = reinterpret_cast<const float4*>(beta);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = lane + 64 * i;
    if (q < C4) {
      const float4 g = g4[q], b = b4[q];
      yr[q] = make_float4((v[i].x - mean) * rstd * g.x + b.x, (v[i].y - mean) * rstd * g.y + b.y,
                          (v[i].z - mean) * rstd * g.z + b.z, (v[i].w - mean) * rstd * g.w + b.w);
    }
  }
  if (lane == 0 && stats) stats[row] = make_float2(mean, rstd);
}

template <int NQ>
__global__ __launch_bounds__(64 * kRowsPerBlock) void ln_bwd_kernel(const float* __restrict__ x,
                                                                    const float* __restrict__ dy,
                                                                    const float* __restrict__ gamma,
                                                                    const float2* __restrict__ stats, long long rows,
                                                                    int C, const float* __restrict__ dres,
                                                                    float* __restrict__ dx) {
  const long long row = (long long)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63, C4 = C >> 2;
  const float2 st = stats[row];
  const float mean = st.x, rstd = st.y;
  const float4* xr = reinterpret_cast<const float4*>(x + row * C);
  const float4* dr = reinterpret_cast<const float4*>(dy + row * C);
  const float4* g4 = reinterpret_cast<const float4*>(gamma);
  float4 xh[NQ], g[NQ];
  float sg = 0.0f, sgx = 0.0f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = lane + 64 * i;
    if (q < C4) {
      const float4 a = xr[q], d = dr[q], w = g4[q];
      xh[i] = make_float4((a.x - mean) * rstd, (a.y - mean) * rstd, (a.z - mean) * rstd, (a.w - mean) * rstd);
      g[i] = make_float4(d.x * w.x, d.y * w.y, d.z * w.z, d.w * w.w);
    } else {
      xh[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      g[i] = xh[i];
    }
    sg += (g[i].x + g[i].y) + (g[i].z + g[i].w);
    sgx += (g[i].x * xh[i].x + g[i].y * xh[i].y) + (g[i].z * xh[i].z + g[i].w * xh[i].w);
  }
  const float mg = wave_sum(sg) / (float)C, mgx = wave_sum(sgx) / (float)C;
  float4* o = reinterpret_cast<float4*>(dx + row * C);
  const float4* rr = reinterpret_cast<const float4*>(dres + row * C);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = lane + 64 * i;
    if (q < C4) {
      float4 v = make_float4(rstd * (g[i].x - mg - xh[i].x * mgx), rstd * (g[i].y - mg - xh[i].y * mgx),
                             rstd * (g[i].z - mg - xh[i].z * mgx), rstd * (g[i].w - mg - xh[i].w * mgx));
      if (dres) {   // the autograd engine's sum of the two gradients, in one pass
        const float4 a = rr[q];
        v = make_float4(v.x + a.x, v.y + a.y, v.z + a.z, v.w + a.w);
      }
      o[q] = v;
    }
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int skp_layernorm_fwd(const float* x, const float* gamma, const float* beta, long long rows, int C,
                                 float eps, float* y, float* stats, void* stream) {
  SKP_CHECK_ARG(x && gamma && beta && y, "null pointer");
  SKP_CHECK_ARG(rows > 0 && C > 0, "non-positive shape");
  SKP_CHECK_ARG(C % 4 == 0 && C <= 2048, "C must be a multiple of 4, at most 2048");
  SKP_CHECK_ARG((rows + kRowsPerBlock - 1) / kRowsPerBlock <= 0x7fffffffLL, "too many rows");
  SKP_CHECK_ARG(aligned16(x) && aligned16(gamma) && aligned16(beta) && aligned16(y) &&
                    (reinterpret_cast<uintptr_t>(stats) & 7) == 0,
                "tensors must be 16-byte aligned (stats 8)");
  const dim3 grid((unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock));
  hipStream_t st = as_stream(stream);
  float2* S = reinterpret_cast<float2*>(stats);
  const int nq = (C / 4 + 63) / 64;
#define SKP_LNF(Q) \
  hipLaunchKernelGGL((ln_fwd_kernel<Q>), grid, dim3(64 * kRowsPerBlock), 0, st, x, gamma, beta, rows, C, eps, y, S)
  if (nq <= 1) SKP_LNF(1);
  else if (nq <= 2) SKP_LNF(2);
  else if (nq <= 4) SKP_LNF(4);
  else SKP_LNF(8);
#undef SKP_LNF
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_layernorm_bwd_add(const float* x, const float* dy, const float* gamma, const float* stats,
                                     long long rows, int C, const float* dres, float* dx, void* stream) {
  SKP_CHECK_ARG(x && dy && gamma && stats && dx, "null pointer");
  SKP_CHECK_ARG(!dres || aligned16(dres), "dres must be 16-byte aligned");
  SKP_CHECK_ARG(rows > 0 && C > 0, "non-positive shape");
  SKP_CHECK_ARG(C % 4 == 0 && C <= 2048, "C must be a multiple of 4, at most 2048");
  SKP_CHECK_ARG((rows + kRowsPerBlock - 1) / kRowsPerBlock <= 0x7fffffffLL, "too many rows");
  SKP_CHECK_ARG(aligned16(x) && aligned16(dy) && aligned16(gamma) && aligned16(dx) &&
                    (reinterpret_cast<uintptr_t>(stats) & 7) == 0,
                "tensors must be 16-byte aligned (stats 8)");
  const dim3 grid((unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock));
  hipStream_t st = as_stream(stream);
  const float2* S = reinterpret_cast<const float2*>(stats);
  const int nq = (C / 4 + 63) / 64;
#define SKP_LNB(Q) \
  hipLaunchKernelGGL((ln_bwd_kernel<Q>), grid, dim3(64 * kRowsPerBlock), 0, st, x, dy, gamma, S, rows, C, dres, dx)
  if (nq <= 1) SKP_LNB(1);
  else if (nq <= 2) SKP_LNB(2);
  else if (nq <= 4) SKP_LNB(4);
  else SKP_LNB(8);
#undef SKP_LNB
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_layernorm_bwd(const float* x, const float* dy, const float* gamma, const float* stats, long long rows,
                                 int C, float* dx, void* stream) {
  return skp_layernorm_bwd_add(x, dy, gamma, stats, rows, C, nullptr, dx, stream);
}
