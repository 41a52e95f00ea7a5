// UNet-side: diffusers GEGLU (FeedForward's first layer, proj → chunk(2) → x · gelu(gate)) as one
// pass each way on gfx950.  PyTorch runs the forward as gelu over the strided gate view plus a
// multiply (two passes and a (rows, I) temporary), and the backward as gelu_backward, two
// multiplies and a concatenation; here the forward reads the projection once and writes the
// output once, and the backward reads dout and the projection once and writes the gradient of
// the projection (both halves) once.  GELU is the exact (erf) form, in torch's expression order.
#include "skp_common.h"

using namespace skp;

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float gelu(float g) { return 0.5f * g * (1.0f + erff(g * 0.70710678118654752440f)); }

__device__ __forceinline__ float gelu_grad(float g) {
  const float kAlpha = 1.12837916709551257390f * 0.70710678118654752440f * 0.5f;   // M_2_SQRTPI·M_SQRT1_2·½
  const float cdf = 0.5f * (1.0f + erff(g * 0.70710678118654752440f));
  const float pdf = expf(-0.5f * g * g) * kAlpha;
  return cdf + g * pdf;
}

// h (rows, 2I) → out (rows, I) = h[:, :I] · gelu(h[:, I:]); float4 lanes (I % 4 == 0)
__global__ __launch_bounds__(kThreads) void geglu_fwd_kernel(const float* __restrict__ h, long long rows, int I,
                                                              float* __restrict__ out) {
  const int q4 = I / 4;
  const long long total = rows * q4;
  for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < total;
       e += (long long)gridDim.x * kThreads) {
    const long long r = e / q4;
    const int j = (int)(e - r * q4) * 4;
    const float4 x = *reinterpret_cast<const float4*>(h + r * 2 * I + j);
    const float4 g = *reinterpret_cast<const float4*>(h + r * 2 * I + I + j);
    *reinterpret_cast<float4*>(out + r * I + j) = make_float4(x.x * gelu(g.x), x.y * gelu(g.y), x.z * gelu(g.z),
                                                              x.w * gelu(g.w));
  }
}

// dh[:, :I] = dout · gelu(g), dh[:, I:] = dout · x · gelu'(g)
__global__ __launch_bounds__(kThreads) void geglu_bwd_kernel(const float* __restrict__ h,
                                                              const float* __restrict__ dout, long long rows, int I,
                                                              float* __restrict__ dh) {
  const int q4 = I / 4;
  const long long total = rows * q4;
  for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < total;
       e += (long long)gridDim.x * kThreads) {
    const long long r = e / q4;
    const int j = (int)(e - r * q4) * 4;
    const float4 x = *reinterpret_cast<const float4*>(h + r * 2 * I + j);
    const float4 g = *reinterpret_cast<const float4*>(h + r * 2 * I + I + j);
    const float4 d = *reinterpret_cast<const float4*>(dout + r * I + j);
    *reinterpret_cast<float4*>(dh + r * 2 * I + j) =
        make_float4(d.x * gelu(g.x), d.y * gelu(g.y), d.z * gelu(g.z), d.w * gelu(g.w));
    *reinterpret_cast<float4*>(dh + r * 2 * I + I + j) =
        make_float4(d.x * x.x * gelu_grad(g.x), d.y * x.y * gelu_grad(g.y), d.z * x.z * gelu_grad(g.z),
                    d.w * x.w * gelu_grad(g.w));
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

unsigned grid_for(long long total) {
  const long long b = (total + kThreads - 1) / kThreads;
  return (unsigned)(b < 8192 ? b : 8192);
}

}  // namespace

extern "C" int skp_geglu_fwd(const float* h, long long rows, int I, float* out, void* stream) {
  SKP_CHECK_ARG(h && out, "null pointer");
  SKP_CHECK_ARG(rows > 0 && I > 0 && I % 4 == 0, "rows > 0 and I a positive multiple of 4");
  SKP_CHECK_ARG(aligned16(h) && aligned16(out), "tensors must be 16-byte aligned");
  hipLaunchKernelGGL(geglu_fwd_kernel, dim3(grid_for(rows * I / 4)), dim3(kThreads), 0, as_stream(stream), h, rows,
                     I, out);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_geglu_bwd(const float* h, const float* dout, long long rows, int I, float* dh, void* stream) {
  SKP_CHECK_ARG(h && dout && dh, "null pointer");
  SKP_CHECK_ARG(rows > 0 && I > 0 && I % 4 == 0, "rows > 0 and I a positive multiple of 4");
  SKP_CHECK_ARG(aligned16(h) && aligned16(dout) && aligned16(dh), "tensors must be 16-byte aligned");
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3(grid_for(rows * I / 4)), dim3(kThreads), 0, as_stream(stream), h, dout,
                     rows, I, dh);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
