// UNet-side: fused softmax backward of the frozen UNet's attention (diffusers-0.8.0
// CrossAttention, the math path softmax(q kᵀ·scale) v) on gfx950.
//
// For each row of P = softmax(S) and its gradient dP:  dS = alpha · P ⊙ (dP − Σ_j P_j dP_j),
// written over dP.  PyTorch runs this as a product pass, a reduction pass and the scale
// multiply of baddbmm's backward (three passes over the 64²-token layers' (B·H, 4096, 4096)
// fp32 tensors, 4.3 GB each at batch 8); here it is one read of P and dP and one write.
// A row is owned by one wave (≤ 1024 columns) or one 256 / 1024-thread workgroup and stays in
// registers between the reduction and the update.
#include "skp_common.h"

using namespace skp;

namespace {

template <int TPR, int EPT, bool VEC>   // threads per row, elements per thread, float4 path (EPT % 4 == 0)
__global__ __launch_bounds__(TPR) void softmax_bwd_kernel(const float* __restrict__ P, float* __restrict__ G,
                                                          long long rows, int cols, float alpha) {
  __shared__ float sred[TPR / WAVE];
  const long long row = blockIdx.x;
  if (row >= rows) return;
  const float* p = P + row * cols;
  float* g = G + row * cols;
  static_assert(!VEC || EPT % 4 == 0, "float4 path needs EPT % 4 == 0");
  float pv[EPT], gv[EPT];
  float dot = 0.0f;
  if (VEC) {
#pragma unroll
    for (int q = 0; q < EPT / 4; ++q) {
      const int e = 4 * (threadIdx.x + q * TPR);
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (e < cols) {
        a = *reinterpret_cast<const float4*>(p + e);
        b = *reinterpret_cast<const float4*>(g + e);
      }
      pv[4 * q] = a.x; pv[4 * q + 1] = a.y; pv[4 * q + 2] = a.z; pv[4 * q + 3] = a.w;
      gv[4 * q] = b.x; gv[4 * q + 1] = b.y; gv[4 * q + 2] = b.z; gv[4 * q + 3] = b.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = threadIdx.x + q * TPR;
      pv[q] = e < cols ? p[e] : 0.0f;
      gv[q] = e < cols ? g[e] : 0.0f;
    }
  }
#pragma unroll
  for (int q = 0; q < EPT; ++q) dot += pv[q] * gv[q];
  dot = wave_sum(dot);
  if (TPR > WAVE) {
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    if (lane == 0) sred[wid] = dot;
    __syncthreads();
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < TPR / WAVE; ++w) t += sred[w];
    dot = t;
  }
  if (VEC) {
#pragma unroll
    for (int q = 0; q < EPT / 4; ++q) {
      const int e = 4 * (threadIdx.x + q * TPR);
      if (e < cols)
        *reinterpret_cast<float4*>(g + e) =
            make_float4(alpha * (pv[4 * q] * (gv[4 * q] - dot)), alpha * (pv[4 * q + 1] * (gv[4 * q + 1] - dot)),
                        alpha * (pv[4 * q + 2] * (gv[4 * q + 2] - dot)),
                        alpha * (pv[4 * q + 3] * (gv[4 * q + 3] - dot)));
    }
  } else {
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = threadIdx.x + q * TPR;
      if (e < cols) g[e] = alpha * (pv[q] * (gv[q] - dot));
    }
  }
}

// In-place row softmax, torch order: m = max, e = exp(x − m), y = e / Σe.  A row stays in
// registers between the two reductions: one read and one write of S.
template <int TPR, int EPT>   // float4 lanes: EPT % 4 == 0
__global__ __launch_bounds__(TPR) void softmax_fwd_kernel(float* __restrict__ S, long long rows, int cols) {
  __shared__ float sred[2][TPR / WAVE];
  const long long row = blockIdx.x;
  if (row >= rows) return;
  float* p = S + row * cols;
  float v[EPT];
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < EPT / 4; ++q) {
    const int e = 4 * (threadIdx.x + q * TPR);
    float4 a = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    if (e < cols) a = *reinterpret_cast<const float4*>(p + e);
    v[4 * q] = a.x;
    v[4 * q + 1] = a.y;
    v[4 * q + 2] = a.z;
    v[4 * q + 3] = a.w;
    m = fmaxf(m, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
  }
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  m = wave_max(m);
  if (TPR > WAVE) {
    if (lane == 0) sred[0][wid] = m;
    __syncthreads();
    float t = sred[0][0];
#pragma unroll
    for (int w = 1; w < TPR / WAVE; ++w) t = fmaxf(t, sred[0][w]);
    m = t;
  }
  float sum = 0.0f;
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    v[q] = expf(v[q] - m);
    sum += v[q];
  }
  sum = wave_sum(sum);
  if (TPR > WAVE) {
    if (lane == 0) sred[1][wid] = sum;
    __syncthreads();
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < TPR / WAVE; ++w) t += sred[1][w];
    sum = t;
  }
#pragma unroll
  for (int q = 0; q < EPT / 4; ++q) {
    const int e = 4 * (threadIdx.x + q * TPR);
    if (e < cols)
      *reinterpret_cast<float4*>(p + e) =
          make_float4(v[4 * q] / sum, v[4 * q + 1] / sum, v[4 * q + 2] / sum, v[4 * q + 3] / sum);
  }
}

}  // namespace

extern "C" int skp_softmax_fwd(float* S, long long rows, int cols, void* stream) {
  SKP_CHECK_ARG(S, "null pointer");
  SKP_CHECK_ARG(rows > 0 && cols > 0, "non-positive shape");
  SKP_CHECK_ARG(cols <= 16384 && cols % 4 == 0, "cols must be a multiple of 4, at most 16384");
  SKP_CHECK_ARG(rows <= 0x7fffffffLL, "too many rows");
  SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(S) & 15) == 0, "S must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)rows);
#define SKP_SF(T, E) hipLaunchKernelGGL((softmax_fwd_kernel<T, E>), grid, dim3(T), 0, st, S, rows, cols)
  if (cols <= 64 * 4) SKP_SF(64, 4);
  else if (cols <= 64 * 8) SKP_SF(64, 8);
  else if (cols <= 64 * 16) SKP_SF(64, 16);
  else if (cols <= 256 * 16) SKP_SF(256, 16);
  else SKP_SF(1024, 16);
#undef SKP_SF
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_softmax_bwd(const float* P, float* dP, long long rows, int cols, float alpha, void* stream) {
  SKP_CHECK_ARG(P && dP, "null pointer");
  SKP_CHECK_ARG(rows > 0 && cols > 0, "non-positive shape");
  SKP_CHECK_ARG(cols <= 16384, "rows longer than 16384 are not supported");
  SKP_CHECK_ARG(rows <= 0x7fffffffLL, "too many rows");
  const bool aligned = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(dP)) & 15) == 0;
  const bool vec = aligned && (cols % 4 == 0);
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)rows);
#define SKP_SB(T, E, V) \
  hipLaunchKernelGGL((softmax_bwd_kernel<T, E, V>), grid, dim3(T), 0, st, P, dP, rows, cols, alpha)
  if (vec) {   // float4 per lane: up to 16 elements per thread
    if (cols <= 64 * 4) SKP_SB(64, 4, true);
    else if (cols <= 64 * 8) SKP_SB(64, 8, true);
    else if (cols <= 64 * 16) SKP_SB(64, 16, true);
    else if (cols <= 256 * 16) SKP_SB(256, 16, true);
    else SKP_SB(1024, 16, true);
  } else {
    if (cols <= 64 * 2) SKP_SB(64, 2, false);
    else if (cols <= 64 * 8) SKP_SB(64, 8, false);
    else if (cols <= 64 * 16) SKP_SB(64, 16, false);
    else if (cols <= 256 * 16) SKP_SB(256, 16, false);
    else SKP_SB(1024, 16, false);
  }
#undef SKP_SB
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
