// A12: affine warp (affine_grid + grid_sample, bilinear, zeros, align_corners=False) and the
// equivariance loss, forward and backward, for gfx950.
//
// Reference: invertable_transform.py:38-92 (RandomAffineWithInverse __call__/inverse) and
// optimize.py:157-163 (equivariance_loss).  Grid coordinates follow ATen: base
// linspace(-1,1,n)·(n-1)/n, grid = [x, y, 1]·θᵀ, unnormalise ((g+1)·n − 1)/2, taps
// nw/ne/sw/se with ATen's weight formulas; out-of-range taps contribute 0.
#include "skp_common.h"

using namespace skp;

namespace {

struct Bilin {
  int x0, y0;
  float w[4];  // nw, ne, sw, se
};

// Rounding follows torch-CPU exactly (the reference warps images on the CPU, optimize.py:386, and
// its goldens are CPU runs): affine_grid's bmm of [x, y, 1] by θᵀ rounds as
// fma(y, θ1, x·θ0) + θ2 (measured against F.affine_grid: bit-equal on every grid point), the CPU
// grid sampler unnormalises as fma(g + 1, n/2, −0.5) and forms the bilinear weights from
// w = ix − floor(ix), e = 1 − w (nw = s·e, ne = s·w, sw = n·e, se = n·w), and the sample as
// ((v_nw·nw + v_ne·ne) + v_sw·sw) + v_se·se without fused multiply-adds.
__device__ __forceinline__ Bilin grid_point(const float* th, int y, int x, int H, int W) {
  const float bx = affine_base(x, W), by = affine_base(y, H);
  const float gx = __fadd_rn(__fmaf_rn(by, th[1], __fmul_rn(bx, th[0])), th[2]);
  const float gy = __fadd_rn(__fmaf_rn(by, th[4], __fmul_rn(bx, th[3])), th[5]);
  const float ix = __fmaf_rn(__fadd_rn(gx, 1.0f), (float)W * 0.5f, -0.5f);
  const float iy = __fmaf_rn(__fadd_rn(gy, 1.0f), (float)H * 0.5f, -0.5f);
  const float x0 = floorf(ix), y0 = floorf(iy);
  const float we = __fsub_rn(ix, x0), ee = __fsub_rn(1.0f, we);   // distance to the west / east side
  const float wn = __fsub_rn(iy, y0), ws = __fsub_rn(1.0f, wn);   // distance to the north / south side
  Bilin b;
  b.x0 = (int)x0;
  b.y0 = (int)y0;
  b.w[0] = __fmul_rn(ws, ee);
  b.w[1] = __fmul_rn(ws, we);
  b.w[2] = __fmul_rn(wn, ee);
  b.w[3] = __fmul_rn(wn, we);
  return b;
}

__device__ __forceinline__ float sample(const float* __restrict__ p, const Bilin& b, int H, int W) {
  float out = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int xx = b.x0 + (k & 1), yy = b.y0 + (k >> 1);
    const float v = (xx >= 0 && xx < W && yy >= 0 && yy < H) ? p[yy * W + xx] : 0.0f;
    out = k == 0 ? __fmul_rn(v, b.w[0]) : __fadd_rn(out, __fmul_rn(v, b.w[k]));
  }
  return out;
}

__device__ __forceinline__ void scatter(float* __restrict__ p, const Bilin& b, int H, int W, float g) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int xx = b.x0 + (k & 1), yy = b.y0 + (k >> 1);
    if (xx >= 0 && xx < W && yy >= 0 && yy < H) atomicAdd(p + yy * W + xx, b.w[k] * g);
  }
}

__global__ void warp_fwd_kernel(const float* __restrict__ x, int B, int C, int H, int W, const float* __restrict__ theta,
                                float* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t HW = (size_t)H * W;
  if (e >= (size_t)B * HW) return;
  const int b = e / HW, p = e % HW;
  const Bilin g = grid_point(theta + 6 * b, p / W, p % W, H, W);
  for (int c = 0; c < C; ++c) {
    const size_t plane = ((size_t)b * C + c) * HW;
    out[plane + p] = sample(x + plane, g, H, W);
  }
}

__global__ void warp_bwd_kernel(const float* __restrict__ gout, int B, int C, int H, int W,
                                const float* __restrict__ theta, float* __restrict__ gin) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t HW = (size_t)H * W;
  if (e >= (size_t)B * HW) return;
  const int b = e / HW, p = e % HW;
  const Bilin g = grid_point(theta + 6 * b, p / W, p % W, H, W);
  for (int c = 0; c < C; ++c) {
    const size_t plane = ((size_t)b * C + c) * HW;
    scatter(gin + plane, g, H, W, gout[plane + p]);
  }
}

constexpr int kThreads = 256;
constexpr int kRowThreads = 1024;   // one workgroup per map row

// rows of image b = [b·seg, (b + 1)·seg) warp with th[6b …] (and, backward, scale by gout[b])
__global__ __launch_bounds__(kRowThreads) void equiv_fwd_kernel(const float* __restrict__ A, const float* __restrict__ At,
                                                             int seg, int h, int w, const float* __restrict__ th,
                                                             double* __restrict__ partial) {
  __shared__ double sd[kRowThreads / 64];
  const int t = blockIdx.x;
  th += 6 * (t / seg);
  const size_t HW = (size_t)h * w;
  const float* a = A + t * HW;
  const float* at = At + t * HW;
  double acc = 0.0;
  for (int p = threadIdx.x; p < (int)HW; p += kRowThreads) {
    const float d = a[p] - sample(at, grid_point(th, p / w, p % w, h, w), h, w);
    acc += (double)(d * d);
  }
  acc = block_sum(acc, sd);
  if (threadIdx.x == 0) partial[t] = acc;
}

__global__ void equiv_bwd_kernel(const float* __restrict__ A, const float* __restrict__ At, int T, int seg, int h,
                                 int w, const float* __restrict__ th, const float* __restrict__ gout, float norm,
                                 float* __restrict__ dA, float* __restrict__ dAt) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t HW = (size_t)h * w;
  if (e >= (size_t)T * HW) return;
  const int t = e / HW, p = e % HW;
  const Bilin g = grid_point(th + 6 * (t / seg), p / w, p % w, h, w);
  const float d = A[e] - sample(At + t * HW, g, h, w);
  const float gd = (d * norm) * gout[t / seg];
  if (dA) dA[e] = gd;
  scatter(dAt + t * HW, g, h, w, -gd);
}

// blockIdx.x = image: out[b] = Σ partial[b·n …] / numel (fixed order; one block per image)
__global__ void finalize_mean_kernel(const double* __restrict__ partial, int n, double numel, float* __restrict__ out) {
  __shared__ double sd[kThreads / 64];
  partial += (size_t)blockIdx.x * n;
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partial[i];
  acc = block_sum(acc, sd);
  if (threadIdx.x == 0) out[blockIdx.x] = (float)(acc / numel);
}

}  // namespace

extern "C" int skp_affine_warp(const float* x, int B, int C, int H, int W, const float* theta, float* out,
                               void* stream) {
  SKP_CHECK_ARG(x && theta && out, "null pointer");
  SKP_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0, "non-positive shape");
  const size_t total = (size_t)B * H * W;
  hipLaunchKernelGGL(warp_fwd_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), x, B, C, H, W, theta,
                     out);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_affine_warp_bwd(const float* gout, int B, int C, int H, int W, const float* theta, float* gin,
                                   void* stream) {
  SKP_CHECK_ARG(gout && theta && gin, "null pointer");
  SKP_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0, "non-positive shape");
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(gin, 0, (size_t)B * C * H * W * sizeof(float), st) != hipSuccess) {
    set_error("skp_affine_warp_bwd: memset failed");
    return SKP_ELAUNCH;
  }
  const size_t total = (size_t)B * H * W;
  hipLaunchKernelGGL(warp_bwd_kernel, dim3((total + 255) / 256), dim3(256), 0, st, gout, B, C, H, W, theta, gin);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_equiv_fwd_batch(const float* A, const float* At, int nb, int T, int h, int w,
                                   const float* theta_inv, double* partial, float* loss, void* stream) {
  SKP_CHECK_ARG(A && At && theta_inv && partial && loss, "null pointer");
  SKP_CHECK_ARG(nb > 0 && T > 0 && h > 0 && w > 0, "non-positive shape");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(equiv_fwd_kernel, dim3(nb * T), dim3(kRowThreads), 0, st, A, At, T, h, w, theta_inv, partial);
  SKP_LAUNCH_CHECK();
  hipLaunchKernelGGL(finalize_mean_kernel, dim3(nb), dim3(kThreads), 0, st, partial, T, (double)T * h * w, loss);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_equiv_fwd(const float* A, const float* At, int T, int h, int w, const float* theta_inv,
                             double* partial, float* loss, void* stream) {
  return skp_equiv_fwd_batch(A, At, 1, T, h, w, theta_inv, partial, loss, stream);
}

extern "C" int skp_equiv_bwd_batch(const float* A, const float* At, int nb, int T, int h, int w,
                                   const float* theta_inv, const float* gout, float* dA, float* dAt, void* stream) {
  SKP_CHECK_ARG(A && At && theta_inv && gout && dAt, "null pointer");
  SKP_CHECK_ARG(nb > 0 && T > 0 && h > 0 && w > 0, "non-positive shape");
  hipStream_t st = as_stream(stream);
  const size_t total = (size_t)nb * T * h * w;
  if (hipMemsetAsync(dAt, 0, total * sizeof(float), st) != hipSuccess) {
    set_error("skp_equiv_bwd: memset failed");
    return SKP_ELAUNCH;
  }
  const float norm = (float)(2.0 / ((double)T * h * w));
  hipLaunchKernelGGL(equiv_bwd_kernel, dim3((total + 255) / 256), dim3(256), 0, st, A, At, nb * T, T, h, w, theta_inv,
                     gout, norm, dA, dAt);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_equiv_bwd(const float* A, const float* At, int T, int h, int w, const float* theta_inv,
                             const float* gout, float* dA, float* dAt, void* stream) {
  return skp_equiv_bwd_batch(A, At, 1, T, h, w, theta_inv, gout, dA, dAt, stream);
}
