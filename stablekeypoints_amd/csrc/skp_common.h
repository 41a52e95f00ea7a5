// Shared device/host helpers for libskp (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string>

#include "../../include/skp.h"

namespace skp {

constexpr int WAVE = 64;

// ------------------------------------------------------------------ host-side error plumbing
void set_error(const std::string& msg);

#define SKP_CHECK_ARG(cond, msg)                 \
  do {                                           \
    if (!(cond)) {                               \
      ::skp::set_error(std::string(__func__) + ": " + (msg)); \
      return SKP_EBADARG;                        \
    }                                            \
  } while (0)

#define SKP_LAUNCH_CHECK()                                                            \
  do {                                                                                \
    hipError_t e_ = hipGetLastError();                                                \
    if (e_ != hipSuccess) {                                                           \
      ::skp::set_error(std::string(__func__) + ": launch failed: " + hipGetErrorString(e_)); \
      return SKP_ELAUNCH;                                                             \
    }                                                                                 \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------ wave reductions (64 lanes)
// Full-wave float reductions without LDS: two quad_perm DPP steps and the half-row / row
// mirrors reduce each 16-lane row, then v_permlane16_swap / v_permlane32_swap (gfx950) exchange
// rows.  Every lane ends with the same bits (each step combines the same two partials).
template <int CTRL>
__device__ __forceinline__ float dpp_read(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <class Op>
__device__ __forceinline__ float wave_reduce(float v, Op op) {
  v = op(v, dpp_read<0xB1>(v));    // quad_perm [1,0,3,2]
  v = op(v, dpp_read<0x4E>(v));    // quad_perm [2,3,0,1]
  v = op(v, dpp_read<0x141>(v));   // row_half_mirror
  v = op(v, dpp_read<0x140>(v));   // row_mirror
  float w = v;
  // the swaps read registers a VALU just wrote: 2 wait states inside the asm (s_nop 1)
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(v), "+v"(w));
  v = op(v, w);
  w = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(v), "+v"(w));
  return op(v, w);
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce(v, [](float a, float b) { return fmaxf(a, b); });
}
__device__ __forceinline__ float wave_sum(float v) {
  return wave_reduce(v, [](float a, float b) { return a + b; });
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// torch.argmax order: NaN beats everything; among equals (or NaNs) the lower index wins.
__device__ __forceinline__ bool argmax_better(float a, int ia, float b, int ib) {
  const bool na = isnan(a), nb = isnan(b);
  if (na) return !nb || ia < ib;
  if (nb) return false;
  return a > b || (a == b && ia < ib);
}

__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(v, o, 64);
    int oi = __shfl_xor(i, o, 64);
    if (argmax_better(ov, oi, v, i)) { v = ov; i = oi; }
  }
}

// Block-wide argmax for blockDim.x = 64*k threads; scratch needs 2*(blockDim/64) words.
__device__ __forceinline__ void block_argmax(float& v, int& i, float* sv, int* si) {
  wave_argmax(v, i);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) { sv[wid] = v; si[wid] = i; }
  __syncthreads();
  if (wid == 0) {
    v = lane < nw ? sv[lane] : -INFINITY;
    i = lane < nw ? si[lane] : 0x7fffffff;
    wave_argmax(v, i);
    if (lane == 0) { sv[0] = v; si[0] = i; }
  }
  __syncthreads();
  v = sv[0];
  i = si[0];
  __syncthreads();
}

__device__ __forceinline__ double block_sum(double v, double* sd) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) sd[wid] = v;
  __syncthreads();
  if (wid == 0) {
    v = lane < nw ? sd[lane] : 0.0;
    v = wave_sum(v);
    if (lane == 0) sd[0] = v;
  }
  __syncthreads();
  v = sd[0];
  __syncthreads();
  return v;
}

__device__ __forceinline__ float block_max(float v, float* sf) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) sf[wid] = v;
  __syncthreads();
  if (wid == 0) {
    v = lane < nw ? sf[lane] : -INFINITY;
    v = wave_max(v);
    if (lane == 0) sf[0] = v;
  }
  __syncthreads();
  v = sf[0];
  __syncthreads();
  return v;
}

// ------------------------------------------------------------------ interpolation taps
// torch upsample_bicubic2d, align_corners=False: src = (dst+0.5)·in/out − 0.5 (unclamped),
// taps floor(src)−1..+2 clamped to [0, in−1], Keys A = −0.75.
struct Taps4 {
  int i[4];     // tap rows/columns, clamped to [0, n_in - 1]
  float w[4];
  int lo;       // first tap before clamping (floor(src) - 1, in [-2, n_in - 2])
};

// The contractions are explicit (the ones the compiler had chosen in every kernel through r04), so
// every kernel — and every inlining context, whatever the SLP vectorizer does — computes the same
// weights bit for bit.
__device__ __forceinline__ float cubic1(float x) {  // |x| <= 1: ((A + 2)·x − (A + 3))·x·x + 1
  const float A = -0.75f;
  return __builtin_fmaf(__builtin_fmaf(A + 2.0f, x, -(A + 3.0f)) * x, x, 1.0f);
}
__device__ __forceinline__ float cubic2(float x) {  // 1 < |x| < 2: ((A·x − 5A)·x + 8A)·x − 4A
  const float A = -0.75f;
  return __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(A, x, -5.0f * A), x, 8.0f * A), x, -4.0f * A);
}

// scale = (float)n_in / (float)n_out, e.g. precomputed on the host (the same IEEE quotient)
__device__ __forceinline__ Taps4 bicubic_taps_s(int dst, int n_in, float scale) {
  const float src = __builtin_fmaf(scale, (float)dst + 0.5f, -0.5f);
  const float f = floorf(src);
  const float t = src - f;
  const int i0 = (int)f;
  Taps4 r;
  r.w[0] = cubic2(t + 1.0f);
  r.w[1] = cubic1(t);
  r.w[2] = cubic1(1.0f - t);
  r.w[3] = cubic2(2.0f - t);
#pragma unroll
  for (int k = 0; k < 4; ++k) r.i[k] = min(max(i0 - 1 + k, 0), n_in - 1);
  r.lo = i0 - 1;
  return r;
}
__device__ __forceinline__ Taps4 bicubic_taps(int dst, int n_in, int n_out) {
  return bicubic_taps_s(dst, n_in, (float)n_in / (float)n_out);
}

// torch bilinear, align_corners=False: src = max((dst+0.5)·in/out − 0.5, 0), upper tap clamped.
struct Taps2 {
  int i0, i1;
  float w0, w1;
};
__device__ __forceinline__ Taps2 bilinear_taps(int dst, int n_in, int n_out) {
  const float scale = (float)n_in / (float)n_out;
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  src = src < 0.0f ? 0.0f : src;
  Taps2 r;
  r.i0 = (int)src;
  r.i1 = r.i0 + (r.i0 < n_in - 1 ? 1 : 0);
  r.w1 = src - (float)r.i0;
  r.w0 = 1.0f - r.w1;
  return r;
}

// affine_grid base coordinate (align_corners=False): linspace(-1, 1, n)[i] * (n-1)/n, with
// linspace rounded as torch-CPU's kernel does (measured bit-equal against torch.linspace for
// n = 100, 128, 512): fma(i, step, −1) for the first half, fma(−(n−1−i), step, 1) for the second.
__device__ __forceinline__ float affine_base(int i, int n) {
  if (n <= 1) return 0.0f;
  const float step = __fdiv_rn(2.0f, (float)(n - 1));
  const float lin = (i < n / 2) ? __fmaf_rn((float)i, step, -1.0f) : __fmaf_rn(-(float)(n - 1 - i), step, 1.0f);
  return __fdiv_rn(__fmul_rn(lin, (float)(n - 1)), (float)n);  // ATen: range * (n - 1) / n
}

// Correctly rounded float sqrt via double (exact for finite floats).
__device__ __forceinline__ float sqrt_rn(float x) { return (float)sqrt((double)x); }

}  // namespace skp
