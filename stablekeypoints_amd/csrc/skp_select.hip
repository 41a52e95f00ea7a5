// A4-A10: argmax family, Gaussian targets, token selection (KL / entropy ranking,
// furthest-point sampling) for gfx950.
//
// Reference: eval.py:39-155 (find_max_pixel, find_k_max_pixels, mask_radius,
// pixel_from_weighted_avg), optimize_token.py:204-242 (gaussian_circle(s)),
// ptp_utils.py:86-187 (find_top_k_gaussian, furthest_point_sampling, entropy_sort).
// Every map row is reduced by one 256-thread workgroup (4 waves) with shuffle
// reductions; index outputs follow torch.argmax (first occurrence, NaN is max) and the
// reference's strict '>' first-wins loops, so they are bit-exact on identical maps.
#include <algorithm>

#include "skp_common.h"

using namespace skp;

namespace {

constexpr int kThreads = 256;      // elementwise kernels
constexpr int kRowThreads = 1024;  // one workgroup per map row (16 waves: a 128² row is 4 float4 per thread)
constexpr int kMaxSubjects = 16;

// Visit a row's elements in increasing index order per thread (16-B loads when aligned).
template <class F>
__device__ __forceinline__ void for_row(const float* __restrict__ m, int HW, F&& f) {
  if ((HW & 3) == 0 && (reinterpret_cast<uintptr_t>(m) & 15) == 0) {
    const float4* m4 = reinterpret_cast<const float4*>(m);
    for (int q = threadIdx.x; q < (HW >> 2); q += blockDim.x) {
      const float4 v = m4[q];
      f(4 * q, v.x);
      f(4 * q + 1, v.y);
      f(4 * q + 2, v.z);
      f(4 * q + 3, v.w);
    }
  } else {
    for (int e = threadIdx.x; e < HW; e += blockDim.x) f(e, m[e]);
  }
}

// Scan one row for its argmax (torch order).  Applies the cumulative radius masks of
// previously found points (eval.mask_radius multiplies by 0/1, so NaN/inf survive as NaN).
__device__ void row_argmax_masked(const float* __restrict__ m, int h, int w, const float* pr, const float* pc,
                                  int nmask, float radius2, float& best, int& bi, float* sv, int* si) {
  best = -INFINITY;
  bi = 0x7fffffff;
  for_row(m, h * w, [&](int e, float v) {
    if (nmask) {
      const float x = (float)(e % w), y = (float)(e / w);
      for (int q = 0; q < nmask; ++q) {
        const float dx = x - pc[q], dy = y - pr[q];
        v = v * ((dx * dx + dy * dy > radius2) ? 1.0f : 0.0f);
      }
    }
    if (argmax_better(v, e, best, bi)) { best = v; bi = e; }
  });
  block_argmax(best, bi, sv, si);
}

__global__ __launch_bounds__(kRowThreads) void argmax_kernel(const float* __restrict__ maps, int T, int h, int w,
                                                          const long long* __restrict__ rows, int seg_len,
                                                          float* __restrict__ pos, long long* __restrict__ idx) {
  __shared__ float sv[kRowThreads / 64];
  __shared__ int si[kRowThreads / 64];
  // with row ids, block i reads row rows[i] of map stack i / seg_len (T rows each)
  const long long row = rows ? rows[blockIdx.x] : blockIdx.x;
  const long long seg = rows ? (long long)(blockIdx.x / seg_len) : 0;
  if (row < 0 || row >= T) {  // invalid row id: poison the output instead of reading out of bounds
    if (threadIdx.x == 0) {
      if (pos) { pos[2 * blockIdx.x] = NAN; pos[2 * blockIdx.x + 1] = NAN; }
      if (idx) idx[blockIdx.x] = -1;
    }
    return;
  }
  float best;
  int bi;
  row_argmax_masked(maps + (seg * T + row) * (long long)h * w, h, w, nullptr, nullptr, 0, 0.0f, best, bi, sv, si);
  if (threadIdx.x == 0) {
    if (pos) {
      pos[2 * blockIdx.x] = (float)(bi / w) + 0.5f;
      pos[2 * blockIdx.x + 1] = (float)(bi % w) + 0.5f;
    }
    if (idx) idx[blockIdx.x] = bi;
  }
}

__global__ __launch_bounds__(kRowThreads) void kmax_kernel(const float* __restrict__ maps, int T, int h, int w, int num,
                                                        float radius2, float* __restrict__ pos,
                                                        float* __restrict__ masked) {
  __shared__ float sv[kRowThreads / 64];
  __shared__ int si[kRowThreads / 64];
  __shared__ float pr[kMaxSubjects], pc[kMaxSubjects];
  const int row = blockIdx.x;
  const float* m = maps + (size_t)row * h * w;
  for (int q = 0; q < num; ++q) {
    float best;
    int bi;
    row_argmax_masked(m, h, w, pr, pc, q, radius2, best, bi, sv, si);
    if (threadIdx.x == 0) {
      pr[q] = (float)(bi / w) + 0.5f;
      pc[q] = (float)(bi % w) + 0.5f;
      pos[((size_t)q * T + row) * 2] = pr[q];
      pos[((size_t)q * T + row) * 2 + 1] = pc[q];
    }
    __syncthreads();
  }
  if (masked) {
    const int HW = h * w;
    for (int e = threadIdx.x; e < HW; e += blockDim.x) {
      float v = m[e];
      const float x = (float)(e % w), y = (float)(e / w);
      for (int q = 0; q < num; ++q) {
        const float dx = x - pc[q], dy = y - pr[q];
        v = v * ((dx * dx + dy * dy > radius2) ? 1.0f : 0.0f);
      }
      masked[(size_t)row * HW + e] = v;
    }
  }
}

__global__ void mask_radius_kernel(const float* __restrict__ maps, int T, int h, int w,
                                   const float* __restrict__ pos, float radius2, float* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t HW = (size_t)h * w;
  if (e >= (size_t)T * HW) return;
  const int t = e / HW, p = e % HW;
  const float dx = (float)(p % w) - pos[2 * t + 1], dy = (float)(p / w) - pos[2 * t];
  out[e] = maps[e] * ((dx * dx + dy * dy > radius2) ? 1.0f : 0.0f);
}

__global__ __launch_bounds__(kRowThreads) void weighted_avg_kernel(float* __restrict__ maps, int h, int w,
                                                                float distance, int mutate, float* __restrict__ pos) {
  __shared__ float sv[kRowThreads / 64];
  __shared__ int si[kRowThreads / 64];
  __shared__ double sd[kRowThreads / 64];
  float* m = maps + (size_t)blockIdx.x * h * w;
  float best;
  int bi;
  row_argmax_masked(m, h, w, nullptr, nullptr, 0, 0.0f, best, bi, sv, si);
  const float r = (float)(bi / w), c = (float)(bi % w);
  const bool cut = distance >= 0.0f;
  const int HW = h * w;
  double tot = 0.0;
  for (int e = threadIdx.x; e < HW; e += blockDim.x) {
    const float x = (float)(e / w), y = (float)(e % w);
    const float dx = x - r, dy = y - c;
    const bool drop = cut && (sqrt_rn(dx * dx + dy * dy) > distance);
    float v = m[e];
    if (drop) {
      v = 0.0f;
      if (mutate) m[e] = 0.0f;
    }
    tot += (double)v;
  }
  tot = block_sum(tot, sd);
  const float denom = (float)tot + 1e-6f;
  double xs = 0.0, ys = 0.0;
  for (int e = threadIdx.x; e < HW; e += blockDim.x) {
    const float x = (float)(e / w), y = (float)(e % w);
    const float dx = x - r, dy = y - c;
    const bool drop = cut && (sqrt_rn(dx * dx + dy * dy) > distance);
    const float v = drop ? 0.0f : m[e];
    const float nv = v / denom;
    xs += (double)(x * nv);
    ys += (double)(y * nv);
  }
  xs = block_sum(xs, sd);
  ys = block_sum(ys, sd);
  if (threadIdx.x == 0) {
    pos[2 * blockIdx.x] = (float)xs + 0.5f;
    pos[2 * blockIdx.x + 1] = (float)ys + 0.5f;
  }
}

// gaussian_circle (optimize_token.py:211-223), averaged over subjects (226-242)
__device__ __forceinline__ float gauss_at(int i, int j, const float* p0, const float* p1, int num, float two_sig2) {
  float acc = 0.0f;
  for (int q = 0; q < num; ++q) {
    const float dj = ((float)j + 0.5f) - p1[q];
    const float di = ((float)i + 0.5f) - p0[q];
    const float d2 = dj * dj + di * di;
    acc += expf(-d2 / two_sig2);
  }
  return acc / (float)num;
}

__global__ void gaussian_target_kernel(const float* __restrict__ pos, int num, int T, int size, float two_sig2,
                                       float* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t S2 = (size_t)size * size;
  if (e >= (size_t)T * S2) return;
  const int t = e / S2, p = e % S2;
  float p0[kMaxSubjects], p1[kMaxSubjects];
  for (int q = 0; q < num; ++q) {
    p0[q] = pos[((size_t)q * T + t) * 2] * (float)size;
    p1[q] = pos[((size_t)q * T + t) * 2 + 1] * (float)size;
  }
  out[e] = gauss_at(p / size, p % size, p0, p1, num, two_sig2);
}

// KL(target ‖ softmax(map + eps)) per token (ptp_utils.py:97-108)
__global__ __launch_bounds__(kRowThreads) void kl_gauss_kernel(const float* __restrict__ maps, int h, int w, int num,
                                                            float radius2, float two_sig2, float eps,
                                                            double* __restrict__ kl) {
  __shared__ float sv[kRowThreads / 64];
  __shared__ int si[kRowThreads / 64];
  __shared__ double sd[kRowThreads / 64];
  __shared__ float sf[kRowThreads / 64];
  __shared__ float pr[kMaxSubjects], pc[kMaxSubjects];
  const float* m = maps + (size_t)blockIdx.x * h * w;
  for (int q = 0; q < num; ++q) {
    float best;
    int bi;
    row_argmax_masked(m, h, w, pr, pc, q, radius2, best, bi, sv, si);
    if (threadIdx.x == 0) {
      pr[q] = (float)(bi / w) + 0.5f;
      pc[q] = (float)(bi % w) + 0.5f;
    }
    __syncthreads();
  }
  // target centres: (find_k_max_pixels / image_h) * size, size = image_h
  float p0[kMaxSubjects], p1[kMaxSubjects];
  for (int q = 0; q < num; ++q) {
    p0[q] = (pr[q] / (float)h) * (float)h;
    p1[q] = (pc[q] / (float)h) * (float)h;
  }
  const int HW = h * w;
  float mx = -INFINITY;
  for_row(m, HW, [&](int, float v) { mx = fmaxf(mx, v + eps); });
  mx = block_max(mx, sf);
  double se = 0.0, sg = 0.0;
  for_row(m, HW, [&](int e, float v) {
    se += (double)expf((v + eps) - mx);
    sg += (double)(gauss_at(e / w, e % w, p0, p1, num, two_sig2) + eps);
  });
  se = block_sum(se, sd);
  sg = block_sum(sg, sd);
  const float sef = (float)se, sgf = (float)sg;
  double acc = 0.0;
  for_row(m, HW, [&](int e, float v) {
    const float P = expf((v + eps) - mx) / sef;
    const float tg = (gauss_at(e / w, e % w, p0, p1, num, two_sig2) + eps) / sgf;
    acc += (double)tg * ((double)logf(tg) - (double)logf(P));
  });
  acc = block_sum(acc, sd);
  if (threadIdx.x == 0) kl[blockIdx.x] = acc;
}

// kl_gauss_kernel with the row resident in registers: one 16-B load per float4 the thread owns
// (the multi-pass kernel streams the 64-KB row four times), and exp((v+eps)−max) and the target
// kept from the Σ pass for the KL pass.  Each thread visits its elements in for_row's order
// (float4 q = tid + j·1024) with the same float operations and the same double accumulation
// order, and the block reductions are the same: bit-identical KL values.  HW ≤ 4·NV·1024, 16-B
// aligned rows with HW % 4 == 0 (the launcher checks); blockIdx.x = row of a (rows, HW) stack,
// so several images' maps are one launch.
template <int NV>
__global__ __launch_bounds__(kRowThreads) void kl_gauss_reg_kernel(const float* __restrict__ maps, int h, int w,
                                                                int num, float radius2, float two_sig2, float eps,
                                                                double* __restrict__ kl) {
  __shared__ float sv[kRowThreads / 64];
  __shared__ int si[kRowThreads / 64];
  __shared__ double sd[kRowThreads / 64];
  __shared__ float sf[kRowThreads / 64];
  __shared__ float pr[kMaxSubjects], pc[kMaxSubjects];
  const int HW = h * w, nq = HW >> 2;
  const float4* m4 = reinterpret_cast<const float4*>(maps + (size_t)blockIdx.x * HW);
  float4 v[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = threadIdx.x + j * kRowThreads;
    v[j] = q < nq ? m4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto visit = [&](auto&& f) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int q = threadIdx.x + j * kRowThreads;
      if (q < nq) {
        f(j, 0, 4 * q, v[j].x);
        f(j, 1, 4 * q + 1, v[j].y);
        f(j, 2, 4 * q + 2, v[j].z);
        f(j, 3, 4 * q + 3, v[j].w);
      }
    }
  };
  for (int q = 0; q < num; ++q) {   // find_k_max_pixels with the cumulative radius masks
    float best = -INFINITY;
    int bi = 0x7fffffff;
    visit([&](int, int, int e, float x) {
      if (q) {
        const float cx = (float)(e % w), cy = (float)(e / w);
        for (int p = 0; p < q; ++p) {
          const float dx = cx - pc[p], dy = cy - pr[p];
          x = x * ((dx * dx + dy * dy > radius2) ? 1.0f : 0.0f);
        }
      }
      if (argmax_better(x, e, best, bi)) { best = x; bi = e; }
    });
    block_argmax(best, bi, sv, si);
    if (threadIdx.x == 0) {
      pr[q] = (float)(bi / w) + 0.5f;
      pc[q] = (float)(bi % w) + 0.5f;
    }
    __syncthreads();
  }
  float p0[kMaxSubjects], p1[kMaxSubjects];
  for (int q = 0; q < num; ++q) {
    p0[q] = (pr[q] / (float)h) * (float)h;
    p1[q] = (pc[q] / (float)h) * (float)h;
  }
  float mx = -INFINITY;
  visit([&](int, int, int, float x) { mx = fmaxf(mx, x + eps); });
  mx = block_max(mx, sf);
  float ex[NV][4], tg[NV][4];
  double se = 0.0, sg = 0.0;
  visit([&](int j, int c, int e, float x) {
    ex[j][c] = expf((x + eps) - mx);
    tg[j][c] = gauss_at(e / w, e % w, p0, p1, num, two_sig2) + eps;
    se += (double)ex[j][c];
    sg += (double)tg[j][c];
  });
  se = block_sum(se, sd);
  sg = block_sum(sg, sd);
  const float sef = (float)se, sgf = (float)sg;
  double acc = 0.0;
  visit([&](int j, int c, int, float) {
    const float P = ex[j][c] / sef;
    const float t = tg[j][c] / sgf;
    acc += (double)t * ((double)logf(t) - (double)logf(P));
  });
  acc = block_sum(acc, sd);
  if (threadIdx.x == 0) kl[blockIdx.x] = acc;
}

// Block sum of N doubles at once (one pair of barriers for all N); sd holds N·(blockDim/64).
template <int N>
__device__ __forceinline__ void block_sum_n(double (&v)[N], double* sd) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    v[k] = wave_sum(v[k]);
    if (lane == 0) sd[k * nw + wid] = v[k];
  }
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      double x = lane < nw ? sd[k * nw + lane] : 0.0;
      x = wave_sum(x);
      if (lane == 0) sd[k * nw] = x;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = sd[k * nw];
}

// Wave sum of doubles on DPP row steps + the gfx950 permlane swaps (both 32-bit halves moved by the
// same control; every lane ends with the same bits), instead of six LDS-routed shuffles.
template <int CTRL>
__device__ __forceinline__ double dpp_read_d(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_read_d<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_read_d<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_read_d<0x141>(v);   // row_half_mirror
  v += dpp_read_d<0x140>(v);   // row_mirror
  const long long b = __builtin_bit_cast(long long, v);
  int lo = (int)b, hi = (int)(b >> 32), wlo = lo, whi = hi;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3"
               : "+v"(lo), "+v"(wlo), "+v"(hi), "+v"(whi));
  v = __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo) +
      __builtin_bit_cast(double, ((long long)whi << 32) | (unsigned)wlo);
  const long long c = __builtin_bit_cast(long long, v);
  lo = (int)c; hi = (int)(c >> 32); wlo = lo; whi = hi;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3"
               : "+v"(lo), "+v"(wlo), "+v"(hi), "+v"(whi));
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo) +
         __builtin_bit_cast(double, ((long long)whi << 32) | (unsigned)wlo);
}
// Block sum of N doubles for thread 0 only (the wave partials added in wave order, one barrier)
template <int N>
__device__ __forceinline__ void block_sum_to0(double (&v)[N], double* sd) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    v[k] = wave_sum_dpp(v[k]);
    if (lane == 0) sd[k * nw + wid] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      double x = sd[k * nw];
      for (int q = 1; q < nw; ++q) x += sd[k * nw + q];
      v[k] = x;
    }
  }
}

// KL(target ‖ softmax(map + eps)) per token for ONE subject (ptp_utils.py:97-108), one HBM read
// of the row.  With u = fl(v + eps) − max (the softmax's shifted logit), t = g + eps the target
// before normalisation and S_t = Σ t, S_e = Σ exp(u):
//   KL = Σ (t/S_t)(log(t/S_t) − (u − log S_e)) = (Σ t·log t − Σ t·u)/S_t − log S_t + log S_e.
// The Gaussian g (optimize_token.py:211-223, σ from the caller) is centred on the row's argmax;
// outside a (2·wr + 1)² window around it g < ulp(eps)/2, so t == eps exactly in fp32 there (the
// host picks wr from σ and eps) and those pixels enter only through Σ u and their count.  So per
// pixel the row costs one exp (for S_e); the Gaussian, its logs and the t·u products run over the
// window only (≈33² pixels at σ = 2, re-read from L2).  Agrees with the per-pixel kernel above to
// fp32 rounding (≈3e-7 absolute on KL ≈ 5, tests/test_gpu_parity.py); rows of HW ≤ 4·NV·BT
// floats, 16-B aligned, HW % 4 == 0 (the launcher checks); blockIdx.x = row of a (rows, HW) stack.
template <int BT, int NV>
__global__ __launch_bounds__(BT) void kl_gauss_win_kernel(const float* __restrict__ maps, int h, int w, float two_sig2,
                                                         float eps, int wr, double* __restrict__ kl) {
  __shared__ float sv[BT / 64];
  __shared__ int si[BT / 64];
  __shared__ double sd[6 * (BT / 64)];
  const int HW = h * w, nq = HW >> 2;
  const float* row = maps + (size_t)blockIdx.x * HW;
  const float4* m4 = reinterpret_cast<const float4*>(row);
  float4 v[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = threadIdx.x + j * BT;
    v[j] = q < nq ? m4[q] : make_float4(0.f, 0.f, 0.f, 0.f);   // cached: the window re-reads hit L2
  }
  // torch.argmax of the row (find_k_max_pixels, num = 1): within a thread the indices increase,
  // so a strict '>' (or the first NaN) keeps the first occurrence
  float best = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = threadIdx.x + j * BT;
    if (q < nq) {
      const float x[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (x[c] > best || (isnan(x[c]) && !isnan(best))) { best = x[c]; bi = 4 * q + c; }
    }
  }
  block_argmax(best, bi, sv, si);
  const float mx = best + eps;   // max of fl(v + eps): rounding is monotonic
  // Σ exp(u) and Σ u: each float4's four terms summed in fp32 (pairwise), the float4 partials in
  // fp64.  exp(u) = exp2(u·log2e) on v_exp_f32: u ≤ 0 and, for attention maps (values in [0, 1]),
  // u ≥ −1 − eps, where the product's rounding and v_exp_f32's ≤ 1-ulp error keep each term within
  // ≈2e-7 relative; the KL ranking's gaps are ≥ 1e-5 on the goldens (tests/test_gpu_parity.py)
  double acc[2] = {0.0, 0.0};
  constexpr float L2E = 1.4426950408889634f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = threadIdx.x + j * BT;
    if (q < nq) {
      const float u0 = (v[j].x + eps) - mx, u1 = (v[j].y + eps) - mx;
      const float u2 = (v[j].z + eps) - mx, u3 = (v[j].w + eps) - mx;
      const float e0 = __builtin_amdgcn_exp2f(u0 * L2E), e1 = __builtin_amdgcn_exp2f(u1 * L2E);
      const float e2 = __builtin_amdgcn_exp2f(u2 * L2E), e3 = __builtin_amdgcn_exp2f(u3 * L2E);
      acc[0] += (double)((e0 + e1) + (e2 + e3));
      acc[1] += (double)((u0 + u1) + (u2 + u3));
    }
  }
  // the target window (find_k_max_pixels / image_h, times size = image_h, as gaussian_circles)
  const float p0 = (((float)(bi / w) + 0.5f) / (float)h) * (float)h;
  const float p1 = (((float)(bi % w) + 0.5f) / (float)h) * (float)h;
  const int c0 = (int)floorf(p0), c1 = (int)floorf(p1);
  const int i0 = max(0, c0 - wr), i1 = min(h - 1, c0 + wr);
  const int j0 = max(0, c1 - wr), j1 = min(w - 1, c1 + wr);
  const int ww = j1 - j0 + 1, nW = (i1 - i0 + 1) * ww;
  double win[4] = {0.0, 0.0, 0.0, 0.0};   // Σ_W t, Σ_W t·log t, Σ_W t·u, Σ_W u
  for (int k = threadIdx.x; k < nW; k += BT) {
    const int i = i0 + k / ww, jj = j0 + k % ww;
    const float di = ((float)i + 0.5f) - p0, dj = ((float)jj + 0.5f) - p1;
    const float t = expf(-(dj * dj + di * di) / two_sig2) + eps;
    const float u = (row[i * w + jj] + eps) - mx;
    win[0] += (double)t;
    win[1] += (double)t * (double)logf(t);
    win[2] += (double)t * (double)u;
    win[3] += (double)u;
  }
  double red[6] = {acc[0], acc[1], win[0], win[1], win[2], win[3]};
  block_sum_n<6>(red, sd);
  if (threadIdx.x == 0) {
    const double e = (double)eps, nO = (double)(HW - nW);
    const double St = red[2] + nO * e;
    const double Stl = red[3] + (nO > 0.0 ? nO * e * (double)logf(eps) : 0.0);
    const double Stu = red[4] + e * (red[1] - red[5]);
    kl[blockIdx.x] = (Stl - Stu) / St - log(St) + log(red[0]);
  }
}

// r05: kl_gauss_win_kernel's arithmetic streamed instead of held: each thread walks its float4s in
// chunks of UNR with a running max of fl(v + eps) and Σ exp relative to it (rescaled by one exp2 when
// a chunk raises the max; threads combine as Σ s_t·exp(m_t − M)), Σ fl(v + eps) for Σu = Σx − HW·M,
// and the argmax as before.  ≈40 VGPRs instead of 83 (the row in registers), so a 128² row's block
// of 4 waves fits 8 per CU and a pass's 4 × 500 rows run in one wave of blocks: the maps stream at
// HBM rate.  Same window terms, same closed form; the sums round differently from the held form
// (Σu by ≤ HW·ulp ≈ 1e-3 absolute, entering KL scaled by eps/S_t ≈ 4e-7: ≈ 1e-10), indices
// bit-exact on the goldens (tests/test_gpu_parity.py).
template <int BT, int UNR>
__global__ __launch_bounds__(BT) void kl_gauss_stream_kernel(const float* __restrict__ maps, int h, int w,
                                                            float two_sig2, float eps, int wr,
                                                            double* __restrict__ kl) {
  __shared__ float sv[BT / 64];
  __shared__ int si[BT / 64];
  __shared__ double sd[6 * (BT / 64)];
  constexpr float L2E = 1.4426950408889634f;
  const int HW = h * w, nq = HW >> 2;
  const float* row = maps + (size_t)blockIdx.x * HW;
  const float4* m4 = reinterpret_cast<const float4*>(row);
  float best = -INFINITY;
  int bi = 0x7fffffff;
  float m = -INFINITY;      // running max of fl(v + eps) over this thread's elements
  double se = 0.0, sx = 0.0;  // Σ exp(x − m) (relative to the running m), Σ x
  for (int q0 = threadIdx.x; q0 < nq; q0 += BT * UNR) {
    float4 v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int q = q0 + k * BT;
      v[k] = q < nq ? m4[q] : make_float4(NAN, NAN, NAN, NAN);
    }
    float cm = -INFINITY;
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int q = q0 + k * BT;
      if (q < nq) {
        const float x[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (x[c] > best || (isnan(x[c]) && !isnan(best))) { best = x[c]; bi = 4 * q + c; }
          cm = fmaxf(cm, x[c] + eps);
        }
      }
    }
    if (cm > m) {   // the chunk raised the running max: rescale the sum once
      se *= (double)__builtin_amdgcn_exp2f((m - cm) * L2E);
      m = cm;
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int q = q0 + k * BT;
      if (q < nq) {
        const float x0 = v[k].x + eps, x1 = v[k].y + eps, x2 = v[k].z + eps, x3 = v[k].w + eps;
        const float e0 = __builtin_amdgcn_exp2f((x0 - m) * L2E), e1 = __builtin_amdgcn_exp2f((x1 - m) * L2E);
        const float e2 = __builtin_amdgcn_exp2f((x2 - m) * L2E), e3 = __builtin_amdgcn_exp2f((x3 - m) * L2E);
        se += (double)((e0 + e1) + (e2 + e3));
        sx += (double)((x0 + x1) + (x2 + x3));
      }
    }
  }
  block_argmax(best, bi, sv, si);
  // the running maxima's maximum is fl(max v + eps) (rounding is monotonic): the argmax reduction
  // already carries it (a NaN row: mx is NaN, so is every sum, as in the held form)
  const float mx = best + eps;
  se *= (double)__builtin_amdgcn_exp2f((m - mx) * L2E);   // m = −inf (no elements): 0 · 0
  const float p0 = (((float)(bi / w) + 0.5f) / (float)h) * (float)h;
  const float p1 = (((float)(bi % w) + 0.5f) / (float)h) * (float)h;
  const int c0 = (int)floorf(p0), c1 = (int)floorf(p1);
  const int i0 = max(0, c0 - wr), i1 = min(h - 1, c0 + wr);
  const int j0 = max(0, c1 - wr), j1 = min(w - 1, c1 + wr);
  const int ww = j1 - j0 + 1, nW = (i1 - i0 + 1) * ww;
  double win[4] = {0.0, 0.0, 0.0, 0.0};   // Σ_W t, Σ_W t·log t, Σ_W t·u, Σ_W u
  // the window's row values re-read 4 per thread at a time (loads in flight together), then its terms
  // in element order per thread (r05 timing probes, profiles/r05zh_kl_probes.txt: the stream alone
  // 25 µs, + block reductions 4 µs, + this window pass 5 µs); the Gaussian and its log on the
  // hardware exp / log (≤ 2 ulp: KL within 1e-6 of the fp64 oracle, indices bit-exact on the
  // goldens; 34.0 → 33.4 µs)
  for (int k0 = threadIdx.x; k0 < nW; k0 += 4 * BT) {
    float rv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + r * BT;
      rv[r] = k < nW ? row[(i0 + k / ww) * w + j0 + k % ww] : 0.0f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + r * BT;
      if (k < nW) {
        const int i = i0 + k / ww, jj = j0 + k % ww;
        const float di = ((float)i + 0.5f) - p0, dj = ((float)jj + 0.5f) - p1;
        const float t = __expf(-(dj * dj + di * di) / two_sig2) + eps;
        const float u = (rv[r] + eps) - mx;
        win[0] += (double)t;
        win[1] += (double)t * (double)__logf(t);
        win[2] += (double)t * (double)u;
        win[3] += (double)u;
      }
    }
  }
  double red[6] = {se, sx, win[0], win[1], win[2], win[3]};
  block_sum_to0<6>(red, sd);
  if (threadIdx.x == 0) {
    const double e = (double)eps, nO = (double)(HW - nW);
    const double su = red[1] - (double)HW * (double)mx;   // Σ u over the row
    const double St = red[2] + nO * e;
    const double Stl = red[3] + (nO > 0.0 ? nO * e * (double)logf(eps) : 0.0);
    const double Stu = red[4] + e * (su - red[5]);
    kl[blockIdx.x] = (Stl - Stu) / St - log(St) + log(red[0]);
  }
}

// entropy of softmax(map) (ptp_utils.py:179-182; torch Categorical renormalises and clamps)
__global__ __launch_bounds__(kRowThreads) void entropy_kernel(const float* __restrict__ maps, int h, int w,
                                                           double* __restrict__ ent) {
  __shared__ double sd[kRowThreads / 64];
  __shared__ float sf[kRowThreads / 64];
  const float* m = maps + (size_t)blockIdx.x * h * w;
  const int HW = h * w;
  float mx = -INFINITY;
  for_row(m, HW, [&](int, float v) { mx = fmaxf(mx, v); });
  mx = block_max(mx, sf);
  double se = 0.0;
  for_row(m, HW, [&](int, float v) { se += (double)expf(v - mx); });
  se = block_sum(se, sd);
  const float sef = (float)se;
  double ps = 0.0;
  for_row(m, HW, [&](int, float v) { ps += (double)(expf(v - mx) / sef); });
  ps = block_sum(ps, sd);
  const float psf = (float)ps;
  const float lo = 1.1920928955078125e-07f, hi = 1.0f - 1.1920928955078125e-07f;
  double acc = 0.0;
  for_row(m, HW, [&](int, float v) {
    const float p = (expf(v - mx) / sef) / psf;
    const float pcl = fminf(fmaxf(p, lo), hi);
    acc += (double)p * (double)logf(pcl);
  });
  acc = block_sum(acc, sd);
  if (threadIdx.x == 0) ent[blockIdx.x] = -acc;
}

// The first top_k of the ascending order of T double keys (NaN last, ties by index) by ranking: key
// i's position is rank_i = #{j : k_j before k_i} (a strict total order), so out[rank_i] = i for
// rank_i < top_k — a sort's first top_k exactly, with one barrier (r05; the r04 bitonic sort ran
// log²(n) barrier-separated stages of one 1024-thread block per image: 15.9 vs 4.8 µs).  A 16-lane row of a wave counts for one key (each lane over every 16th key, then one DPP
// row sum), so a 256-thread block ranks 16 keys; grid = (images, ⌈T / 16⌉).  The block stages its
// image's T keys (≤ 8192) in LDS.
__global__ __launch_bounds__(256) void rank_topk_kernel(const double* __restrict__ keys, int T, int top_k,
                                                        long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* k = reinterpret_cast<double*>(smem);
  const int b = blockIdx.y;
  keys += (size_t)b * T;
  out += (size_t)b * top_k;
  for (int i = threadIdx.x; i < T; i += blockDim.x) k[i] = keys[i];
  __syncthreads();
  const int li = threadIdx.x & 15;
  const int i = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int ii = min(i, T - 1);
  const double ki = k[ii];
  const bool ni = isnan(ki);
  int r = 0;
  for (int j = li; j < T; j += 16) {
    const double kj = k[j];   // NaN kj compares false: never before a number
    r += ni ? ((!isnan(kj) || j < ii) ? 1 : 0) : ((kj < ki || (kj == ki && j < ii)) ? 1 : 0);
  }
  // Σ over the 16-lane row (integers: exact in any order)
  r += __shfl_xor(r, 1, 16);
  r += __shfl_xor(r, 2, 16);
  r += __shfl_xor(r, 4, 16);
  r += __shfl_xor(r, 8, 16);
  if (li == 0 && i < T && r < top_k) out[r] = i;
}

// r06: the ranking of the KL keys and the candidates' argmax in ONE launch (skp_fps_keys_batch): block
// (i, b) ranks token i among image b's T keys — rank_topk_kernel's strict order (NaN last, ties by
// index), the block's threads over the other keys — and, if the rank r is below C, takes the argmax
// of token i's row of the FPS maps (argmax_kernel's torch order and position convention) and writes
// candidate r.  Ranks are a permutation, so exactly one block writes each candidate; the C blocks
// with an argmax to do are the only ones that read a map row.  The selection chain of a pass is
// KL → (rank + argmax) → FPS.
#ifndef SKP_RANKARG_THREADS
#define SKP_RANKARG_THREADS 512   // threads per rank_argmax block (256: 15.2 us, 1024: 15.8, 512: 13.3)
#endif
constexpr int kRankArgThreads = SKP_RANKARG_THREADS;
__global__ __launch_bounds__(kRankArgThreads) void rank_argmax_kernel(const double* __restrict__ keys, int T, int C,
                                                                   const float* __restrict__ maps, int h, int w,
                                                                   long long* __restrict__ cand,
                                                                   float* __restrict__ pos) {
  __shared__ float sv[kRankArgThreads / 64];
  __shared__ int si[kRankArgThreads / 64];
  __shared__ double sd[kRankArgThreads / 64];
  const int i = blockIdx.x, b = blockIdx.y;
  keys += (size_t)b * T;
  const double ki = keys[i];
  const bool ni = isnan(ki);
  double r = 0.0;   // a count: exact in any order
  for (int j = threadIdx.x; j < T; j += blockDim.x) {
    const double kj = keys[j];   // NaN kj compares false: never before a number
    r += ni ? ((!isnan(kj) || j < i) ? 1.0 : 0.0) : ((kj < ki || (kj == ki && j < i)) ? 1.0 : 0.0);
  }
  const int rank = (int)block_sum(r, sd);
  if (rank >= C) return;   // uniform
  // the row's argmax with 4 16-B loads in flight per thread (argmax_better is a total order, so
  // the visiting order does not matter)
  const float* m = maps + ((size_t)b * T + i) * h * w;
  const int HW = h * w;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  if ((HW & 3) == 0 && (reinterpret_cast<uintptr_t>(m) & 15) == 0) {
    const float4* m4 = reinterpret_cast<const float4*>(m);
    const int n4 = HW >> 2, step = blockDim.x;
    for (int q0 = threadIdx.x; q0 < n4; q0 += 4 * step) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (q0 + u * step < n4) v[u] = m4[q0 + u * step];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = q0 + u * step;
        if (q < n4) {
          if (argmax_better(v[u].x, 4 * q, best, bi)) { best = v[u].x; bi = 4 * q; }
          if (argmax_better(v[u].y, 4 * q + 1, best, bi)) { best = v[u].y; bi = 4 * q + 1; }
          if (argmax_better(v[u].z, 4 * q + 2, best, bi)) { best = v[u].z; bi = 4 * q + 2; }
          if (argmax_better(v[u].w, 4 * q + 3, best, bi)) { best = v[u].w; bi = 4 * q + 3; }
        }
      }
    }
  } else {
    for (int e = threadIdx.x; e < HW; e += blockDim.x)
      if (argmax_better(m[e], e, best, bi)) { best = m[e]; bi = e; }
  }
  block_argmax(best, bi, sv, si);
  if (threadIdx.x == 0) {
    const size_t o = (size_t)b * C + rank;
    cand[o] = i;
    pos[2 * o] = (float)(bi / w) + 0.5f;
    pos[2 * o + 1] = (float)(bi % w) + 0.5f;
  }
}

// Furthest-point sampling over candidate positions (ptp_utils.py:115-159), one wave.
__global__ __launch_bounds__(64) void fps_kernel(const float* __restrict__ cpos, const long long* __restrict__ cand,
                                                 int C, int h, int top_k, long long* __restrict__ out,
                                                 int* __restrict__ n_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* pr = reinterpret_cast<float*>(smem);
  float* pc = pr + C;
  long long* tok = reinterpret_cast<long long*>(pc + C);  // 8·C bytes in: 8-aligned
  long long* sel = tok + C;
  float* spr = reinterpret_cast<float*>(sel + top_k);
  float* spc = spr + top_k;
  const int lane = threadIdx.x;
  cpos += (size_t)blockIdx.x * 2 * C;   // blockIdx.x = image of a batched launch
  cand += (size_t)blockIdx.x * C;
  out += (size_t)blockIdx.x * top_k;
  if (n_out) n_out += blockIdx.x;
  for (int i = lane; i < C; i += 64) {
    pr[i] = cpos[2 * i] / (float)h;
    pc[i] = cpos[2 * i + 1] / (float)h;
    tok[i] = cand[i];
  }
  __syncthreads();
  // 1) furthest pair: reference loops i < j in order with strict '>' (first wins).
  float best = -1.0f;
  long long brank = 0x7fffffffffffffffLL;
  for (int i = lane; i < C; i += 64) {
    for (int j = i + 1; j < C; ++j) {
      const float dr = pr[i] - pr[j], dc = pc[i] - pc[j];
      const float d = sqrt_rn(dr * dr + dc * dc);
      if (d > best) { best = d; brank = (long long)i * C + j; }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const long long orank = __shfl_xor(brank, o, 64);
    if (ob > best || (ob == best && orank < brank)) { best = ob; brank = orank; }
  }
  int nsel = 0;
  if (brank != 0x7fffffffffffffffLL) {
    const int i0 = (int)(brank / C), j0 = (int)(brank % C);
    if (lane == 0) {
      sel[0] = tok[i0]; spr[0] = pr[i0]; spc[0] = pc[i0];
      sel[1] = tok[j0]; spr[1] = pr[j0]; spc[1] = pc[j0];
    }
    nsel = 2;
  }
  __syncthreads();
  // 2) greedy max-min additions (top_k - 2 rounds), candidates skipped if their token is selected
  for (int round = 0; round < top_k - 2 && nsel >= 2; ++round) {
    float bd = -1.0f;
    int bi = 0x7fffffff;
    for (int i = lane; i < C; i += 64) {
      bool taken = false;
      for (int q = 0; q < nsel; ++q) taken |= (sel[q] == tok[i]);
      if (taken) continue;
      float dmin = INFINITY;
      bool nan_seen = false;
      for (int q = 0; q < nsel; ++q) {
        const float dr = pr[i] - spr[q], dc = pc[i] - spc[q];
        const float d = sqrt_rn(dr * dr + dc * dc);
        nan_seen |= isnan(d);
        dmin = fminf(dmin, d);
      }
      if (nan_seen) dmin = NAN;  // torch.min propagates NaN
      if (dmin > bd) { bd = dmin; bi = i; }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(bd, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > bd || (ob == bd && oi < bi)) { bd = ob; bi = oi; }
    }
    if (bi != 0x7fffffff) {
      if (lane == 0) { sel[nsel] = tok[bi]; spr[nsel] = pr[bi]; spc[nsel] = pc[bi]; }
      ++nsel;
    }
    __syncthreads();
  }
  for (int q = lane; q < top_k; q += 64) out[q] = q < nsel ? sel[q] : -1;
  if (lane == 0 && n_out) *n_out = nsel;
}

// The same FPS with one candidate per lane (C ≤ 64, top_k ≤ 64; r06): the candidates' positions and
// tokens stay in registers and every lane keeps its candidate's running minimum distance to the
// selected set, updated with the newest pick only — fminf over the same distances in another order
// is the same minimum, and the NaN flag is an OR — so a round is one distance and one wave
// reduction instead of nsel distances read back from LDS.  Selections are identical to fps_kernel's.
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ long long lane_ll(long long v, int l) {
  const unsigned long long u = (unsigned long long)v;
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return (long long)(((unsigned long long)hi << 32) | lo);
}
// (v, i) with the larger v, ties to the smaller i (FPS's strict '>' in index order; v is never NaN
// here), over the wave: DPP within each 16-lane row (quad perms, half-row and row mirrors — no LDS
// round trip as __shfl_xor's ds_bpermute takes), then the 4 row results read into SGPRs: the result
// is wave-uniform
__device__ __forceinline__ void fps_pick(float& v, int& i, float ov, int oi) {
  if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}
template <int CTRL>
__device__ __forceinline__ void fps_dpp_step(float& v, int& i) {
  const float ov = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v),
                                                                         __builtin_bit_cast(int, v), CTRL, 0xF, 0xF,
                                                                         false));
  const int oi = __builtin_amdgcn_update_dpp(i, i, CTRL, 0xF, 0xF, false);
  fps_pick(v, i, ov, oi);
}
__device__ __forceinline__ void fps_wave_best(float& v, int& i) {
  fps_dpp_step<0xB1>(v, i);    // quad_perm [1, 0, 3, 2]
  fps_dpp_step<0x4E>(v, i);    // quad_perm [2, 3, 0, 1]
  fps_dpp_step<0x141>(v, i);   // row_half_mirror
  fps_dpp_step<0x140>(v, i);   // row_mirror
  float bv = lane_f(v, 0);
  int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
  for (int r = 1; r < 4; ++r) fps_pick(bv, bi, lane_f(v, 16 * r), __builtin_amdgcn_readlane(i, 16 * r));
  v = bv;
  i = bi;
}

__global__ __launch_bounds__(64) void fps_wave_kernel(const float* __restrict__ cpos, const long long* __restrict__ cand,
                                                      int C, int h, int top_k, long long* __restrict__ out,
                                                      int* __restrict__ n_out) {
  const int lane = threadIdx.x;
  cpos += (size_t)blockIdx.x * 2 * C;   // blockIdx.x = image of a batched launch
  cand += (size_t)blockIdx.x * C;
  out += (size_t)blockIdx.x * top_k;
  if (n_out) n_out += blockIdx.x;
  const bool act = lane < C;
  const float pr = act ? cpos[2 * lane] / (float)h : 0.0f;
  const float pc = act ? cpos[2 * lane + 1] / (float)h : 0.0f;
  const long long tk = act ? cand[lane] : 0;
  auto dist = [&](float qr, float qc) {
    const float dr = pr - qr, dc = pc - qc;
    return sqrt_rn(dr * dr + dc * dc);
  };
  // 1) furthest pair: the pairs (lane, j > lane) in j order with strict '>' (first wins)
  float best = -1.0f;
  int brank = 0x7fffffff;
  for (int j = 1; j < C; ++j) {
    const float qr = lane_f(pr, j), qc = lane_f(pc, j);
    if (act && j > lane) {
      const float d = dist(qr, qc);
      if (d > best) { best = d; brank = lane * C + j; }
    }
  }
  fps_wave_best(best, brank);
  long long mine = -1;   // lane q: the q-th selected token
  int nsel = 0;
  float dm = INFINITY;
  bool nan_seen = false, taken = false;
  auto add = [&](int s) {   // candidate s joins the selected set
    const long long ts = lane_ll(tk, s);
    const float qr = lane_f(pr, s), qc = lane_f(pc, s);
    if (lane == nsel) mine = ts;
    ++nsel;
    taken |= tk == ts;
    const float d = dist(qr, qc);
    nan_seen |= isnan(d);
    dm = fminf(dm, d);
  };
  if (brank != 0x7fffffff) {
    add(brank / C);
    add(brank % C);
  }
  // 2) greedy max-min additions (top_k − 2 rounds), candidates skipped if their token is selected
  for (int round = 0; round < top_k - 2 && nsel >= 2; ++round) {
    float bd = -1.0f;
    int bi = 0x7fffffff;
    if (act && !taken) {
      const float v = nan_seen ? NAN : dm;   // torch.min propagates NaN
      if (v > bd) { bd = v; bi = lane; }
    }
    fps_wave_best(bd, bi);
    if (bi == 0x7fffffff) break;   // nothing left: the later rounds find nothing either
    add(bi);
  }
  if (lane < top_k) out[lane] = mine;
  if (lane == 0 && n_out) *n_out = nsel;
}

void launch_fps(const float* cpos, const long long* cand, int nb, int n_cand, int h, int top_k, long long* out,
                int* n_out, hipStream_t st) {
  if (n_cand <= 64 && top_k <= 64) {
    hipLaunchKernelGGL(fps_wave_kernel, dim3(nb), dim3(64), 0, st, cpos, cand, n_cand, h, top_k, out, n_out);
  } else {
    const size_t lds = (size_t)n_cand * 8 + (size_t)n_cand * 8 + (size_t)top_k * 8 + (size_t)top_k * 8;
    hipLaunchKernelGGL(fps_kernel, dim3(nb), dim3(64), lds, st, cpos, cand, n_cand, h, top_k, out, n_out);
  }
}

// ------------------------------------------------------------------------------------ losses
__global__ __launch_bounds__(kRowThreads) void sharpen_fwd_kernel(const float* __restrict__ A, int T, int h, int w,
                                                               int num, float radius2, float two_sig2,
                                                               float* __restrict__ pos, double* __restrict__ partial) {
  __shared__ float sv[kRowThreads / 64];
  __shared__ int si[kRowThreads / 64];
  __shared__ double sd[kRowThreads / 64];
  __shared__ float pr[kMaxSubjects], pc[kMaxSubjects];
  const int row = blockIdx.x;
  const float* m = A + (size_t)row * h * w;
  for (int q = 0; q < num; ++q) {
    float best;
    int bi;
    row_argmax_masked(m, h, w, pr, pc, q, radius2, best, bi, sv, si);
    if (threadIdx.x == 0) {
      pr[q] = (float)(bi / w) + 0.5f;
      pc[q] = (float)(bi % w) + 0.5f;
      // sharpening_loss: pos = find_k_max_pixels(A) / A.shape[-1]
      pos[((size_t)q * T + row) * 2] = pr[q] / (float)w;
      pos[((size_t)q * T + row) * 2 + 1] = pc[q] / (float)w;
    }
    __syncthreads();
  }
  float p0[kMaxSubjects], p1[kMaxSubjects];
  for (int q = 0; q < num; ++q) {
    p0[q] = (pr[q] / (float)w) * (float)h;
    p1[q] = (pc[q] / (float)w) * (float)h;
  }
  double acc = 0.0;
  for_row(m, h * w, [&](int e, float v) {
    const float d = v - gauss_at(e / w, e % w, p0, p1, num, two_sig2);
    acc += (double)(d * d);
  });
  acc = block_sum(acc, sd);
  if (threadIdx.x == 0) partial[row] = acc;
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

// rows of image b = [b·seg, (b + 1)·seg): its loss gradient is gout[b]
__global__ void sharpen_bwd_kernel(const float* __restrict__ A, int T, int seg, int h, int w, int num, float two_sig2,
                                   const float* __restrict__ pos, const float* __restrict__ gout, float norm,
                                   float* __restrict__ dA) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t HW = (size_t)h * w;
  if (e >= (size_t)T * HW) return;
  const int t = e / HW, p = e % HW;
  float p0[kMaxSubjects], p1[kMaxSubjects];
  for (int q = 0; q < num; ++q) {
    p0[q] = pos[((size_t)q * T + t) * 2] * (float)h;
    p1[q] = pos[((size_t)q * T + t) * 2 + 1] * (float)h;
  }
  const float d = A[e] - gauss_at(p / w, p % w, p0, p1, num, two_sig2);
  dA[e] = (d * norm) * gout[t / seg];
}

}  // namespace

// ------------------------------------------------------------------------------------ C ABI
extern "C" int skp_argmax2d(const float* maps, int T, int h, int w, const long long* rows, int n_rows, float* pos,
                            long long* idx, void* stream) {
  SKP_CHECK_ARG(maps && (pos || idx), "null pointer");
  SKP_CHECK_ARG(T > 0 && h > 0 && w > 0, "non-positive shape");
  const int nr = rows ? n_rows : T;
  SKP_CHECK_ARG(nr > 0, "no rows");
  hipLaunchKernelGGL(argmax_kernel, dim3(nr), dim3(kRowThreads), 0, as_stream(stream), maps, T, h, w, rows, nr, pos,
                     idx);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_k_max_pixels(const float* maps, int T, int h, int w, int num, float radius2, float* pos,
                                float* masked, void* stream) {
  SKP_CHECK_ARG(maps && pos, "null pointer");
  SKP_CHECK_ARG(T > 0 && h > 0 && w > 0, "non-positive shape");
  SKP_CHECK_ARG(num >= 1 && num <= kMaxSubjects, "num out of range [1, 16]");
  hipLaunchKernelGGL(kmax_kernel, dim3(T), dim3(kRowThreads), 0, as_stream(stream), maps, T, h, w, num, radius2, pos,
                     masked);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_mask_radius(const float* maps, int T, int h, int w, const float* pos, float radius2, float* out,
                               void* stream) {
  SKP_CHECK_ARG(maps && pos && out, "null pointer");
  SKP_CHECK_ARG(T > 0 && h > 0 && w > 0, "non-positive shape");
  const size_t total = (size_t)T * h * w;
  hipLaunchKernelGGL(mask_radius_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), maps, T, h, w, pos,
                     radius2, out);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_weighted_avg(float* maps, int T, int h, int w, float distance, int mutate, float* pos,
                                void* stream) {
  SKP_CHECK_ARG(maps && pos, "null pointer");
  SKP_CHECK_ARG(T > 0 && h > 0 && w > 0, "non-positive shape");
  hipLaunchKernelGGL(weighted_avg_kernel, dim3(T), dim3(kRowThreads), 0, as_stream(stream), maps, h, w, distance, mutate,
                     pos);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_gaussian_target(const float* pos, int num, int T, int size, float sigma, float* out, void* stream) {
  SKP_CHECK_ARG(pos && out, "null pointer");
  SKP_CHECK_ARG(T > 0 && size > 0, "non-positive shape");
  SKP_CHECK_ARG(num >= 1 && num <= kMaxSubjects, "num out of range [1, 16]");
  const float two_sig2 = (float)(2.0 * (double)sigma * (double)sigma);
  const size_t total = (size_t)T * size * size;
  hipLaunchKernelGGL(gaussian_target_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), pos, num, T,
                     size, two_sig2, out);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

static int launch_sort(const double* keys, int T, int top_k, long long* out, hipStream_t st, int nb = 1) {
  SKP_CHECK_ARG(T <= 8192, "T > 8192 tokens is not supported by the selection ranking");
  hipLaunchKernelGGL(rank_topk_kernel, dim3((T + 15) / 16, nb), dim3(256), (size_t)T * sizeof(double), st, keys, T,
                     top_k, out);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

#ifndef SKP_KL_WIN
#define SKP_KL_WIN 1   // 0: the per-pixel register kernel for one subject too (A/B build)
#endif
#ifndef SKP_KL_REG
#define SKP_KL_REG 1   // 0: the four-pass kl_gauss_kernel for every shape (A/B build)
#endif

extern "C" int skp_topk_gaussian_batch(const float* maps, int nb, int T, int h, int w, int top_k, float sigma,
                                       float epsilon, int num_subjects, long long* out, double* kl, void* workspace,
                                       void* stream) {
  SKP_CHECK_ARG(maps && out && workspace, "null pointer");
  SKP_CHECK_ARG(nb > 0 && T > 0 && h > 0 && w > 0, "non-positive shape");
  SKP_CHECK_ARG(top_k >= 0 && top_k <= T, "top_k out of range");
  SKP_CHECK_ARG(num_subjects >= 1 && num_subjects <= kMaxSubjects, "num_subjects out of range [1, 16]");
  double* keys = kl ? kl : reinterpret_cast<double*>(workspace);
  const double rad = 0.05 * (double)h;
  const float radius2 = (float)(rad * rad);
  const float two_sig2 = (float)(2.0 * (double)sigma * (double)sigma);
  hipStream_t st = as_stream(stream);
  const int rows = nb * T, HW = h * w;
  const bool reg = SKP_KL_REG && (HW & 3) == 0 && (reinterpret_cast<uintptr_t>(maps) & 15) == 0;
  if (reg && SKP_KL_WIN && num_subjects == 1 && HW <= 4 * 16 * 1024) {
    // window half-width: outside it exp(−d²/2σ²) < eps·2⁻²⁵ (< half an ulp of eps), i.e.
    // d² ≥ 2σ²·(ln(1/eps) + 20); no usable bound (eps ≤ 0, σ ≤ 0, …): the whole row
    int wr = h > w ? h : w;
    const double kk = epsilon > 0.0f ? log(1.0 / (double)epsilon) + 20.0 : -1.0;
    if (kk > 0.0 && sigma > 0.0f && isfinite(kk)) {
      const double r = ceil(sqrt((double)two_sig2 * kk));
      if (r < (double)wr) wr = (int)r;
    }
    // rows up to 128²: the streamed form, 256 threads, one float4 per thread per chunk (kbench kl4
    // 39.4 µs vs 40.0–40.9 at two, 42.0 at four, 44.5–44.9 for the held form,
    // profiles/r05zb_kl_stream_ab.txt); larger rows (find_best_indices at 256²): the held form.
    // (Fusing the ranking behind the KL rows — each image's last block ranks — measured 2.5× slower,
    // profiles/r05w_a8_fused_ab.txt, and was removed in r06.)
    if (HW <= 4 * 16 * 256)
      hipLaunchKernelGGL((kl_gauss_stream_kernel<256, 1>), dim3(rows), dim3(256), 0, st, maps, h, w, two_sig2, epsilon, wr,
                         keys);
    else
      hipLaunchKernelGGL((kl_gauss_win_kernel<1024, 16>), dim3(rows), dim3(1024), 0, st, maps, h, w, two_sig2, epsilon,
                         wr, keys);
    SKP_LAUNCH_CHECK();
    if (top_k == 0) return SKP_OK;
    return launch_sort(keys, T, top_k, out, st, nb);
  } else if (reg && HW <= 4 * 1 * kRowThreads)
    hipLaunchKernelGGL(kl_gauss_reg_kernel<1>, dim3(rows), dim3(kRowThreads), 0, st, maps, h, w, num_subjects,
                       radius2, two_sig2, epsilon, keys);
  else if (reg && HW <= 4 * 2 * kRowThreads)
    hipLaunchKernelGGL(kl_gauss_reg_kernel<2>, dim3(rows), dim3(kRowThreads), 0, st, maps, h, w, num_subjects,
                       radius2, two_sig2, epsilon, keys);
  else if (reg && HW <= 4 * 4 * kRowThreads)
    hipLaunchKernelGGL(kl_gauss_reg_kernel<4>, dim3(rows), dim3(kRowThreads), 0, st, maps, h, w, num_subjects,
                       radius2, two_sig2, epsilon, keys);
  else
    hipLaunchKernelGGL(kl_gauss_kernel, dim3(rows), dim3(kRowThreads), 0, st, maps, h, w, num_subjects, radius2,
                       two_sig2, epsilon, keys);
  SKP_LAUNCH_CHECK();
  if (top_k == 0) return SKP_OK;
  return launch_sort(keys, T, top_k, out, st, nb);
}

extern "C" int skp_topk_keys(const double* keys, int nb, int T, int top_k, long long* out, void* stream) {
  SKP_CHECK_ARG(keys && out, "null pointer");
  SKP_CHECK_ARG(nb > 0 && T > 0, "non-positive shape");
  SKP_CHECK_ARG(top_k >= 0 && top_k <= T, "top_k out of range");
  if (top_k == 0) return SKP_OK;
  return launch_sort(keys, T, top_k, out, as_stream(stream), nb);
}

extern "C" int skp_topk_gaussian(const float* maps, int T, int h, int w, int top_k, float sigma, float epsilon,
                                 int num_subjects, long long* out, double* kl, void* workspace, void* stream) {
  return skp_topk_gaussian_batch(maps, 1, T, h, w, top_k, sigma, epsilon, num_subjects, out, kl, workspace, stream);
}

extern "C" int skp_entropy_sort(const float* maps, int T, int h, int w, int top_k, long long* out, double* ent,
                                void* workspace, void* stream) {
  SKP_CHECK_ARG(maps && out && workspace, "null pointer");
  SKP_CHECK_ARG(T > 0 && h > 0 && w > 0, "non-positive shape");
  SKP_CHECK_ARG(top_k >= 0 && top_k <= T, "top_k out of range");
  double* keys = ent ? ent : reinterpret_cast<double*>(workspace);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(entropy_kernel, dim3(T), dim3(kRowThreads), 0, st, maps, h, w, keys);
  SKP_LAUNCH_CHECK();
  if (top_k == 0) return SKP_OK;
  return launch_sort(keys, T, top_k, out, st);
}

extern "C" int skp_fps_batch(const float* maps, int nb, int T, int h, int w, const long long* cand, int n_cand,
                             int top_k, long long* out, int* n_out, void* workspace, void* stream) {
  SKP_CHECK_ARG(maps && cand && out && workspace, "null pointer");
  SKP_CHECK_ARG(nb > 0 && T > 0 && h > 0 && w > 0, "non-positive shape");
  SKP_CHECK_ARG(n_cand >= 2, "furthest_point_sampling needs at least two candidates");
  SKP_CHECK_ARG(n_cand <= 4096, "n_cand > 4096");
  SKP_CHECK_ARG(top_k >= 2 && top_k <= 1024, "top_k out of range [2, 1024]");
  hipStream_t st = as_stream(stream);
  float* cpos = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(argmax_kernel, dim3(nb * n_cand), dim3(kRowThreads), 0, st, maps, T, h, w, cand, n_cand, cpos,
                     (long long*)nullptr);
  SKP_LAUNCH_CHECK();
  SKP_CHECK_ARG((size_t)n_cand * 16 + (size_t)top_k * 16 <= 64 * 1024, "fps LDS budget exceeded");
  launch_fps(cpos, cand, nb, n_cand, h, top_k, out, n_out, st);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_fps_keys_batch(const double* keys, const float* maps, int nb, int T, int h, int w, int n_cand,
                                  int top_k, long long* cand, long long* out, int* n_out, void* workspace,
                                  void* stream) {
  SKP_CHECK_ARG(keys && maps && cand && out && workspace, "null pointer");
  SKP_CHECK_ARG(nb > 0 && T > 0 && h > 0 && w > 0, "non-positive shape");
  SKP_CHECK_ARG(T <= 8192, "T > 8192 tokens is not supported by the selection ranking");
  SKP_CHECK_ARG(n_cand >= 2 && n_cand <= T, "n_cand must be in [2, T]");
  SKP_CHECK_ARG(n_cand <= 4096, "n_cand > 4096");
  SKP_CHECK_ARG(top_k >= 2 && top_k <= 1024, "top_k out of range [2, 1024]");
  SKP_CHECK_ARG(nb <= 65535 && n_cand <= 65535, "grid too large");
  hipStream_t st = as_stream(stream);
  float* cpos = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(rank_argmax_kernel, dim3(T, nb), dim3(kRankArgThreads), 0, st, keys, T, n_cand, maps, h, w, cand, cpos);
  SKP_LAUNCH_CHECK();
  SKP_CHECK_ARG((size_t)n_cand * 16 + (size_t)top_k * 16 <= 64 * 1024, "fps LDS budget exceeded");
  launch_fps(cpos, cand, nb, n_cand, h, top_k, out, n_out, st);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_fps(const float* maps, int T, int h, int w, const long long* cand, int n_cand, int top_k,
                       long long* out, int* n_out, void* workspace, void* stream) {
  return skp_fps_batch(maps, 1, T, h, w, cand, n_cand, top_k, out, n_out, workspace, stream);
}

extern "C" int skp_sharpen_fwd_batch(const float* A, int nb, int T, int h, int w, float sigma, int num_subjects,
                                     float* pos, double* partial, float* loss, void* stream) {
  SKP_CHECK_ARG(A && pos && partial && loss, "null pointer");
  SKP_CHECK_ARG(nb > 0 && T > 0 && h > 0 && w > 0, "non-positive shape");
  SKP_CHECK_ARG(num_subjects >= 1 && num_subjects <= kMaxSubjects, "num_subjects out of range [1, 16]");
  const double rad = 0.05 * (double)h;
  const float radius2 = (float)(rad * rad);
  const float two_sig2 = (float)(2.0 * (double)sigma * (double)sigma);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(sharpen_fwd_kernel, dim3(nb * T), dim3(kRowThreads), 0, st, A, nb * T, h, w, num_subjects, radius2,
                     two_sig2, pos, partial);
  SKP_LAUNCH_CHECK();
  hipLaunchKernelGGL(finalize_mean_kernel, dim3(nb), dim3(kThreads), 0, st, partial, T, (double)T * h * w, loss);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_sharpen_fwd(const float* A, int T, int h, int w, float sigma, int num_subjects, float* pos,
                               double* partial, float* loss, void* stream) {
  return skp_sharpen_fwd_batch(A, 1, T, h, w, sigma, num_subjects, pos, partial, loss, stream);
}

extern "C" int skp_sharpen_bwd_batch(const float* A, int nb, int T, int h, int w, float sigma, int num_subjects,
                                     const float* pos, const float* gout, float* dA, void* stream) {
  SKP_CHECK_ARG(A && pos && gout && dA, "null pointer");
  SKP_CHECK_ARG(nb > 0 && T > 0 && h > 0 && w > 0, "non-positive shape");
  SKP_CHECK_ARG(num_subjects >= 1 && num_subjects <= kMaxSubjects, "num_subjects out of range [1, 16]");
  const float two_sig2 = (float)(2.0 * (double)sigma * (double)sigma);
  const float norm = (float)(2.0 / ((double)T * h * w));
  const size_t total = (size_t)nb * T * h * w;
  hipLaunchKernelGGL(sharpen_bwd_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), A, nb * T, T, h,
                     w, num_subjects, two_sig2, pos, gout, norm, dA);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_sharpen_bwd(const float* A, int T, int h, int w, float sigma, int num_subjects, const float* pos,
                               const float* gout, float* dA, void* stream) {
  return skp_sharpen_bwd_batch(A, 1, T, h, w, sigma, num_subjects, pos, gout, dA, stream);
}
