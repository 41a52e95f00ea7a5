// Fused GroupNorm (+ optional SiLU) forward / input-gradient backward for the frozen SD-1.5
// UNet / VAE (NCHW fp32) on gfx950.  An optional per-(sample, channel) input shift folds the
// preceding convolution's bias and the resnet's time-embedding add into the same passes:
// GroupNorm(x + shift[b, c]) without materialising x + shift.
//
// The hot path's backward runs through the UNet into the token embedding,
// and GroupNorm is the UNet's largest non-GEMM cost (ATen: statistics kernel + separate
// normalise and SiLU passes).  Here a group is one contiguous run of (C/G)·H·W floats:
//   pass 1  per-chunk partial (Σx, Σx²) in fp64          (grid = B·G·nsplit blocks)
//   pass 2  per-chunk: combine the group's partials in fixed order -> mean, rstd;
//           y = act((x − mean)·rstd·γ + β)                (read x once, write y once)
// Backward (parameters are frozen, so only dx): with z = x̂γ + β, gz = dy·act'(z),
//   dx = rstd·(gz·γ − mean(gz·γ) − x̂·mean(gz·γ·x̂))
//   pass 1  per-chunk partial (Σ gzγ, Σ gzγx̂) in fp64;  pass 2  dx.
// All reductions have a fixed order, so results are run-to-run deterministic.
#include <algorithm>

#include "skp_common.h"

using namespace skp;

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 16384;   // floats per block (64 KiB)

#ifndef SKP_GN_FAST
// 1: σ(z) through v_rcp_f32 (1 ulp) instead of the IEEE division sequence, and the channel of a
// group offset by a 32-bit division (the 64-bit one is a ≈40-instruction sequence per float4);
// 0: the r04 forms (A/B build)
#define SKP_GN_FAST 1
#endif
__device__ __forceinline__ float sigmoid_of(float z) {
#if SKP_GN_FAST
  return __builtin_amdgcn_rcpf(1.0f + __expf(-z));
#else
  return 1.0f / (1.0f + __expf(-z));
#endif
}
__device__ __forceinline__ float silu(float z) {
#if SKP_GN_FAST
  return z * sigmoid_of(z);
#else
  return z / (1.0f + __expf(-z));
#endif
}
__device__ __forceinline__ float silu_grad(float z) {
  const float s = sigmoid_of(z);
  return s * (1.0f + z * (1.0f - s));
}

struct GNShape {
  int B, C, G, cpg, nsplit;
  long long HW, len;  // len = cpg * HW (floats per group)
};

// channel (within its group) of float e of a group: e < len < 2^32 (make_shape)
__device__ __forceinline__ int chan_of(long long e, const GNShape& sh) {
#if SKP_GN_FAST
  return (int)((unsigned)e / (unsigned)sh.HW);
#else
  return (int)(e / sh.HW);
#endif
}

#ifndef SKP_GN_BATCH
#define SKP_GN_BATCH 4   // float4s per thread whose loads are issued together (1: one at a time, A/B)
#endif
// This thread's float4s of [lo, hi) (stride 4·kThreads), visited in ascending order (the order the
// per-thread sums depend on) in batches of SKP_GN_BATCH whose loads ld(e) are issued before any
// use(e, v): the small 64² / 32² groups are otherwise one load latency per float4.
template <typename Ld, typename Use>
__device__ __forceinline__ void for_f4(long long lo, long long hi, Ld ld, Use use) {
  constexpr int U = SKP_GN_BATCH;
  constexpr long long S = 4 * kThreads;
  long long e = lo + 4 * threadIdx.x;
  for (; e + (U - 1) * S < hi; e += U * S) {
    decltype(ld(e)) v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld(e + u * S);
#pragma unroll
    for (int u = 0; u < U; ++u) use(e + u * S, v[u]);
  }
  for (; e < hi; e += S) use(e, ld(e));
}

// a + b rounded on its own (never contracted into the product that made a): the fused residual
// gradient equals autograd's separate add bit for bit
__device__ __forceinline__ float add_rn(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}

// x and dy (and the residual gradient, r) of one float4 position (the backward's loads)
struct Pair4 {
  float4 a, b, r;
};
__device__ __forceinline__ Pair4 make_pair4(float4 a, float4 b) { return Pair4{a, b, make_float4(0.f, 0.f, 0.f, 0.f)}; }

// shift of channel c of group grp (nullptr: none)
__device__ __forceinline__ float shift_of(const float* __restrict__ shift, const GNShape& sh, int grp, int c) {
  return shift ? shift[(grp / sh.G) * sh.C + c] : 0.0f;
}

__device__ __forceinline__ void block_sum2(double& a, double& b, double* sd) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sd[2 * wid] = a; sd[2 * wid + 1] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double x = 0.0, y = 0.0;
    for (int w = 0; w < kThreads / 64; ++w) { x += sd[2 * w]; y += sd[2 * w + 1]; }
    sd[0] = x;
    sd[1] = y;
  }
  __syncthreads();
  a = sd[0];
  b = sd[1];
}

template <bool VEC>
__global__ __launch_bounds__(kThreads) void gn_stats_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ shift, GNShape sh,
                                                            double* __restrict__ partial) {
  __shared__ double sd[2 * kThreads / 64];
  const int grp = blockIdx.x / sh.nsplit, sp = blockIdx.x % sh.nsplit;
  const int g = grp % sh.G;
  const float* base = x + (size_t)grp * sh.len;
  const long long lo = (long long)sp * kChunk, hi = min(sh.len, lo + kChunk);
  double s1 = 0.0, s2 = 0.0;
  if (VEC) {
    for_f4(lo, hi, [&](long long e) { return *reinterpret_cast<const float4*>(base + e); },
           [&](long long e, float4 v) {
             const float t = shift_of(shift, sh, grp, g * sh.cpg + chan_of(e, sh));
             v.x += t; v.y += t; v.z += t; v.w += t;
             s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
             s2 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
           });
  } else {
    for (long long e = lo + threadIdx.x; e < hi; e += kThreads) {
      const double v = base[e] + shift_of(shift, sh, grp, g * sh.cpg + chan_of(e, sh));
      s1 += v;
      s2 += v * v;
    }
  }
  block_sum2(s1, s2, sd);
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = s1;
    partial[2 * blockIdx.x + 1] = s2;
  }
}

// Statistics from the producing convolution's epilogue (skp_conv3x3_wino2_gn): part[b][c][seg] =
// (mean, M2) of pixel segment seg (n = HW / nseg pixels) of channel c — computed there around a
// pivot inside the segment, so they carry no cancellation however far the channel's mean is from 0
// (r05; the r04 form stored fp32 (Σx, Σx²) and lost the variance to E[x²] − mean² when
// |mean| ≫ std).  One block per (sample, group), one pass over the group's cpg·nseg
// segments in fp64 with the channel's shift folded into the segment mean: Σ(x+t) = n·(mean + t),
// Σ(x+t)² = M2 + n·(mean + t)² (Chan's combination, exact up to fp64 rounding), then one block
// reduction; the group totals go to chunk 0 of the layout gn_apply_kernel reads (the other chunks
// zero), so the apply pass is the one skp_groupnorm_fwd uses.
__global__ __launch_bounds__(kThreads) void gn_part_combine_kernel(const float2* __restrict__ part, int nseg,
                                                                   const float* __restrict__ shift, GNShape sh,
                                                                   double* __restrict__ partial) {
  __shared__ double sd[2 * kThreads / 64];
  const int grp = blockIdx.x;   // b·G + g
  const int b = grp / sh.G, g = grp - b * sh.G;
  const float2* pg = part + ((size_t)b * sh.C + (size_t)g * sh.cpg) * nseg;
  const double n = (double)(sh.HW / nseg);
  double s1 = 0.0, s2 = 0.0;
  for (int e = threadIdx.x; e < sh.cpg * nseg; e += kThreads) {
    const float2 v = pg[e];
    const double t = shift ? (double)shift[(size_t)b * sh.C + g * sh.cpg + e / nseg] : 0.0;
    const double mt = (double)v.x + t;
    s1 += n * mt;
    s2 += (double)v.y + n * mt * mt;
  }
  block_sum2(s1, s2, sd);
  if (threadIdx.x < sh.nsplit) {
    partial[2 * ((size_t)grp * sh.nsplit + threadIdx.x)] = threadIdx.x == 0 ? s1 : 0.0;
    partial[2 * ((size_t)grp * sh.nsplit + threadIdx.x) + 1] = threadIdx.x == 0 ? s2 : 0.0;
  }
  for (int k = kThreads + threadIdx.x; k < sh.nsplit; k += kThreads) {
    partial[2 * ((size_t)grp * sh.nsplit + k)] = 0.0;
    partial[2 * ((size_t)grp * sh.nsplit + k) + 1] = 0.0;
  }
}

// combine one group's partials (fixed order) -> (mean, rstd)
__device__ __forceinline__ void group_moments(const double* __restrict__ partial, int grp, const GNShape& sh, float eps,
                                              float& mean, float& rstd) {
  double s1 = 0.0, s2 = 0.0;
  for (int k = 0; k < sh.nsplit; ++k) {
    s1 += partial[2 * (grp * sh.nsplit + k)];
    s2 += partial[2 * (grp * sh.nsplit + k) + 1];
  }
  const double n = (double)sh.len;
  const double m = s1 / n;
  double var = s2 / n - m * m;
  var = var < 0.0 ? 0.0 : var;
  mean = (float)m;
  rstd = (float)(1.0 / sqrt(var + (double)eps));
}

template <bool VEC, bool ACT>
__global__ __launch_bounds__(kThreads) void gn_apply_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ shift, GNShape sh, float eps,
                                                            const double* __restrict__ partial, float* __restrict__ y,
                                                            float* __restrict__ stats) {
  __shared__ float sm[2];
  const int grp = blockIdx.x / sh.nsplit, sp = blockIdx.x % sh.nsplit;
  if (threadIdx.x == 0) {
    float mean, rstd;
    group_moments(partial, grp, sh, eps, mean, rstd);
    sm[0] = mean;
    sm[1] = rstd;
    if (sp == 0 && stats) { stats[2 * grp] = mean; stats[2 * grp + 1] = rstd; }
  }
  __syncthreads();
  const float mean = sm[0], rstd = sm[1];
  const int g = grp % sh.G;
  const float* base = x + (size_t)grp * sh.len;
  float* out = y + (size_t)grp * sh.len;
  const long long lo = (long long)sp * kChunk, hi = min(sh.len, lo + kChunk);
  if (VEC) {   // HW % 4 == 0: a float4 never straddles two channels
    for_f4(lo, hi, [&](long long e) { return *reinterpret_cast<const float4*>(base + e); },
           [&](long long e, float4 v) {
             const int c = g * sh.cpg + chan_of(e, sh);
             const float ga = gamma[c] * rstd, be = beta[c] - mean * gamma[c] * rstd;
             const float t = shift_of(shift, sh, grp, c);
             v.x += t; v.y += t; v.z += t; v.w += t;
             v.x = v.x * ga + be; v.y = v.y * ga + be; v.z = v.z * ga + be; v.w = v.w * ga + be;
             if (ACT) { v.x = silu(v.x); v.y = silu(v.y); v.z = silu(v.z); v.w = silu(v.w); }
             *reinterpret_cast<float4*>(out + e) = v;
           });
  } else {
    for (long long e = lo + threadIdx.x; e < hi; e += kThreads) {
      const int c = g * sh.cpg + chan_of(e, sh);
      float v = ((base[e] + shift_of(shift, sh, grp, c)) - mean) * rstd * gamma[c] + beta[c];
      out[e] = ACT ? silu(v) : v;
    }
  }
}

template <bool VEC, bool ACT>
__global__ __launch_bounds__(kThreads) void gn_bwd_stats_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ dy,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                const float* __restrict__ shift, GNShape sh,
                                                                const float* __restrict__ stats,
                                                                double* __restrict__ partial) {
  __shared__ double sd[2 * kThreads / 64];
  const int grp = blockIdx.x / sh.nsplit, sp = blockIdx.x % sh.nsplit;
  const int g = grp % sh.G;
  const float mean = stats[2 * grp], rstd = stats[2 * grp + 1];
  const float* xb = x + (size_t)grp * sh.len;
  const float* db = dy + (size_t)grp * sh.len;
  const long long lo = (long long)sp * kChunk, hi = min(sh.len, lo + kChunk);
  double s1 = 0.0, s2 = 0.0;
  // the elements of x / dy at e0 (n = 4 or 1 of them), in order
  auto body = [&](long long e0, const float* xv, const float* dv, int n) {
    const int c = g * sh.cpg + chan_of(e0, sh);
    const float ga = gamma[c], be = beta[c], t = shift_of(shift, sh, grp, c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= n) break;
      const float xh = ((xv[k] + t) - mean) * rstd;
      float gz = dv[k];
      if (ACT) gz *= silu_grad(xh * ga + be);
      const float gg = gz * ga;
      s1 += (double)gg;
      s2 += (double)gg * (double)xh;
    }
  };
  if (VEC) {
    for_f4(lo, hi,
           [&](long long e) {
             return make_pair4(*reinterpret_cast<const float4*>(xb + e), *reinterpret_cast<const float4*>(db + e));
           },
           [&](long long e, const Pair4& v) {
             const float xv[4] = {v.a.x, v.a.y, v.a.z, v.a.w}, dv[4] = {v.b.x, v.b.y, v.b.z, v.b.w};
             body(e, xv, dv, 4);
           });
  } else {
    for (long long e0 = lo + threadIdx.x; e0 < hi; e0 += kThreads) body(e0, xb + e0, db + e0, 1);
  }
  block_sum2(s1, s2, sd);
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = s1;
    partial[2 * blockIdx.x + 1] = s2;
  }
}

template <bool VEC, bool ACT>
__global__ __launch_bounds__(kThreads) void gn_bwd_apply_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ dy,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                const float* __restrict__ shift, GNShape sh,
                                                                const float* __restrict__ stats,
                                                                const double* __restrict__ partial,
                                                                const float* __restrict__ dres,
                                                                float* __restrict__ dx) {
  __shared__ float sm[2];
  const int grp = blockIdx.x / sh.nsplit, sp = blockIdx.x % sh.nsplit;
  if (threadIdx.x == 0) {
    double s1 = 0.0, s2 = 0.0;
    for (int k = 0; k < sh.nsplit; ++k) {
      s1 += partial[2 * (grp * sh.nsplit + k)];
      s2 += partial[2 * (grp * sh.nsplit + k) + 1];
    }
    sm[0] = (float)(s1 / (double)sh.len);
    sm[1] = (float)(s2 / (double)sh.len);
  }
  __syncthreads();
  const float ma = sm[0], mb = sm[1];
  const int g = grp % sh.G;
  const float mean = stats[2 * grp], rstd = stats[2 * grp + 1];
  const float* xb = x + (size_t)grp * sh.len;
  const float* db = dy + (size_t)grp * sh.len;
  float* ob = dx + (size_t)grp * sh.len;
  const float* rb = dres ? dres + (size_t)grp * sh.len : nullptr;
  const long long lo = (long long)sp * kChunk, hi = min(sh.len, lo + kChunk);
  // dx of the n (4 or 1) elements at e0: xv, dv, av (the residual gradient; 0 without one)
  auto body = [&](long long e0, const float* xv, const float* dv, const float* av, float* r, int n) {
    const int c = g * sh.cpg + chan_of(e0, sh);
    const float ga = gamma[c], be = beta[c], t = shift_of(shift, sh, grp, c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= n) break;
      const float xh = ((xv[k] + t) - mean) * rstd;
      float gz = dv[k];
      if (ACT) gz *= silu_grad(xh * ga + be);
      r[k] = rstd * (gz * ga - ma - xh * mb);
      if (rb) r[k] = add_rn(r[k], av[k]);   // + the gradient of x's other consumer (the residual / shortcut)
    }
  };
  if (VEC) {
    for_f4(lo, hi,
           [&](long long e) {
             Pair4 v = make_pair4(*reinterpret_cast<const float4*>(xb + e), *reinterpret_cast<const float4*>(db + e));
             v.r = rb ? *reinterpret_cast<const float4*>(rb + e) : make_float4(0.f, 0.f, 0.f, 0.f);
             return v;
           },
           [&](long long e, const Pair4& v) {
             const float xv[4] = {v.a.x, v.a.y, v.a.z, v.a.w}, dv[4] = {v.b.x, v.b.y, v.b.z, v.b.w};
             const float av[4] = {v.r.x, v.r.y, v.r.z, v.r.w};
             float r[4];
             body(e, xv, dv, av, r, 4);
             *reinterpret_cast<float4*>(ob + e) = make_float4(r[0], r[1], r[2], r[3]);
           });
  } else {
    for (long long e0 = lo + threadIdx.x; e0 < hi; e0 += kThreads) {
      const float av = rb ? rb[e0] : 0.0f;
      float r;
      body(e0, xb + e0, db + e0, &av, &r, 1);
      ob[e0] = r;
    }
  }
}

// out = a + (h + bias[c]): a convolution's bias add fused into the residual add that
// consumes it (same fp32 rounding order as the two separate torch adds).
template <bool VEC>
__global__ __launch_bounds__(kThreads) void residual_bias_kernel(const float* __restrict__ a,
                                                                 const float* __restrict__ h,
                                                                 const float* __restrict__ bias, int C, long long HW,
                                                                 long long total, float* __restrict__ out) {
  const long long step = (long long)gridDim.x * kThreads * (VEC ? 4 : 1);
  for (long long e = ((long long)blockIdx.x * kThreads + threadIdx.x) * (VEC ? 4 : 1); e < total; e += step) {
    const float b = bias[(e / HW) % C];
    if (VEC) {
      const float4 x = *reinterpret_cast<const float4*>(a + e), y = *reinterpret_cast<const float4*>(h + e);
      *reinterpret_cast<float4*>(out + e) = make_float4(x.x + (y.x + b), x.y + (y.y + b), x.z + (y.z + b),
                                                        x.w + (y.w + b));
    } else {
      out[e] = a[e] + (h[e] + b);
    }
  }
}

bool make_shape(int B, int C, long long HW, int G, GNShape& sh) {
  if (B <= 0 || C <= 0 || HW <= 0 || G <= 0 || C % G != 0) return false;
  sh.B = B; sh.C = C; sh.G = G; sh.cpg = C / G; sh.HW = HW;
  sh.len = (long long)sh.cpg * HW;
  sh.nsplit = (int)((sh.len + kChunk - 1) / kChunk);
  return sh.len < (1LL << 32);   // chan_of's 32-bit offsets
}

}  // namespace

extern "C" int skp_groupnorm_workspace(int B, int C, long long HW, int G) {
  GNShape sh;
  if (!make_shape(B, C, HW, G, sh)) return -1;
  return B * G * sh.nsplit * 2;   // doubles
}

extern "C" int skp_groupnorm_fwd(const float* x, const float* gamma, const float* beta, const float* shift, int B,
                                 int C, long long HW, int G, float eps, int act, float* y, float* stats,
                                 double* partial, void* stream) {
  SKP_CHECK_ARG(x && gamma && beta && y && partial, "null pointer");
  GNShape sh;
  SKP_CHECK_ARG(make_shape(B, C, HW, G, sh), "bad shape (C must be divisible by G)");
  const bool vec = (HW % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(y) & 15) == 0);
  hipStream_t st = as_stream(stream);
  const dim3 grid(B * G * sh.nsplit);
  if (vec) hipLaunchKernelGGL(gn_stats_kernel<true>, grid, dim3(kThreads), 0, st, x, shift, sh, partial);
  else hipLaunchKernelGGL(gn_stats_kernel<false>, grid, dim3(kThreads), 0, st, x, shift, sh, partial);
  SKP_LAUNCH_CHECK();
#define SKP_GN_APPLY(V, A) \
  hipLaunchKernelGGL((gn_apply_kernel<V, A>), grid, dim3(kThreads), 0, st, x, gamma, beta, shift, sh, eps, partial, y, \
                     stats)
  if (vec) { if (act) SKP_GN_APPLY(true, true); else SKP_GN_APPLY(true, false); }
  else { if (act) SKP_GN_APPLY(false, true); else SKP_GN_APPLY(false, false); }
#undef SKP_GN_APPLY
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_groupnorm_fwd_part(const float* x, const float* gamma, const float* beta, const float* shift,
                                      const float* part, int nseg, int B, int C, long long HW, int G, float eps,
                                      int act, float* y, float* stats, double* partial, void* stream) {
  SKP_CHECK_ARG(x && gamma && beta && y && partial && part, "null pointer");
  SKP_CHECK_ARG(nseg > 0 && HW % nseg == 0, "nseg must divide H·W");
  GNShape sh;
  SKP_CHECK_ARG(make_shape(B, C, HW, G, sh), "bad shape (C must be divisible by G)");
  SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(part) & 7) == 0, "part must be 8-byte aligned");
  const bool vec = (HW % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(y) & 15) == 0);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(gn_part_combine_kernel, dim3(B * G), dim3(kThreads), 0, st, reinterpret_cast<const float2*>(part),
                     nseg, shift, sh, partial);
  SKP_LAUNCH_CHECK();
  const dim3 grid(B * G * sh.nsplit);
#define SKP_GN_APPLY(V, A) \
  hipLaunchKernelGGL((gn_apply_kernel<V, A>), grid, dim3(kThreads), 0, st, x, gamma, beta, shift, sh, eps, partial, y, \
                     stats)
  if (vec) { if (act) SKP_GN_APPLY(true, true); else SKP_GN_APPLY(true, false); }
  else { if (act) SKP_GN_APPLY(false, true); else SKP_GN_APPLY(false, false); }
#undef SKP_GN_APPLY
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_groupnorm_bwd_add(const float* x, const float* dy, const float* gamma, const float* beta,
                                     const float* shift, const float* stats, int B, int C, long long HW, int G, int act,
                                     const float* dres, float* dx, double* partial, void* stream) {
  SKP_CHECK_ARG(x && dy && gamma && beta && stats && dx && partial, "null pointer");
  GNShape sh;
  SKP_CHECK_ARG(make_shape(B, C, HW, G, sh), "bad shape (C must be divisible by G)");
  const bool vec = (HW % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(dy) & 15) == 0) && ((reinterpret_cast<uintptr_t>(dx) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(dres) & 15) == 0);
  hipStream_t st = as_stream(stream);
  const dim3 grid(B * G * sh.nsplit);
#define SKP_GN_B(K, V, A, ...) hipLaunchKernelGGL((K<V, A>), grid, dim3(kThreads), 0, st, __VA_ARGS__)
  if (vec) {
    if (act) SKP_GN_B(gn_bwd_stats_kernel, true, true, x, dy, gamma, beta, shift, sh, stats, partial);
    else SKP_GN_B(gn_bwd_stats_kernel, true, false, x, dy, gamma, beta, shift, sh, stats, partial);
  } else {
    if (act) SKP_GN_B(gn_bwd_stats_kernel, false, true, x, dy, gamma, beta, shift, sh, stats, partial);
    else SKP_GN_B(gn_bwd_stats_kernel, false, false, x, dy, gamma, beta, shift, sh, stats, partial);
  }
  SKP_LAUNCH_CHECK();
  if (vec) {
    if (act) SKP_GN_B(gn_bwd_apply_kernel, true, true, x, dy, gamma, beta, shift, sh, stats, partial, dres, dx);
    else SKP_GN_B(gn_bwd_apply_kernel, true, false, x, dy, gamma, beta, shift, sh, stats, partial, dres, dx);
  } else {
    if (act) SKP_GN_B(gn_bwd_apply_kernel, false, true, x, dy, gamma, beta, shift, sh, stats, partial, dres, dx);
    else SKP_GN_B(gn_bwd_apply_kernel, false, false, x, dy, gamma, beta, shift, sh, stats, partial, dres, dx);
  }
#undef SKP_GN_B
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_groupnorm_bwd(const float* x, const float* dy, const float* gamma, const float* beta,
                                 const float* shift, const float* stats, int B, int C, long long HW, int G, int act,
                                 float* dx, double* partial, void* stream) {
  return skp_groupnorm_bwd_add(x, dy, gamma, beta, shift, stats, B, C, HW, G, act, nullptr, dx, partial, stream);
}

extern "C" int skp_residual_bias_add(const float* a, const float* h, const float* bias, int B, int C, long long HW,
                                     float* out, void* stream) {
  SKP_CHECK_ARG(a && h && bias && out, "null pointer");
  SKP_CHECK_ARG(B > 0 && C > 0 && HW > 0, "non-positive shape");
  const long long total = (long long)B * C * HW;
  const bool vec = (HW % 4 == 0) && ((reinterpret_cast<uintptr_t>(a) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(h) & 15) == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  const long long units = vec ? total / 4 : total;
  const int blocks = (int)std::min<long long>((units + kThreads - 1) / kThreads, 256LL * 16);
  hipStream_t st = as_stream(stream);
  if (vec) hipLaunchKernelGGL(residual_bias_kernel<true>, dim3(blocks), dim3(kThreads), 0, st, a, h, bias, C, HW, total, out);
  else hipLaunchKernelGGL(residual_bias_kernel<false>, dim3(blocks), dim3(kThreads), 0, st, a, h, bias, C, HW, total, out);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
