// A1 capture (softmax of bicubic-upsampled cross-attention logits) and A3 aggregate
// (collect_maps) for gfx950.
//
// Reference: ptp_utils.py:508-538 (capture branch of the patched CrossAttention.forward)
// and optimize.py:27-79 (collect_maps).  Design notes in DESIGN.md §Kernels.
//
// Capture works from the layer's low-resolution logits z_low = q kᵀ·scale (s×s pixels):
// bicubic upsampling and to_q are linear, so softmax(to_q(bicubic(x)) kᵀ·scale) =
// softmax(bicubic(z_low)).  One workgroup owns one output row y of one (batch·head) b:
//   1. vertical bicubic pass  V[j][n] = Σ_k wy_k · z_low[b][iy_k·s + j][n]   (LDS, s×N)
//   2. per output pixel x (one wave each): Z[n] = Σ_k wx_k · V[ix_k][n], softmax over n
//      with wave64 shuffle reductions, coalesced store of the (N,) row of attn.
// The backward recomputes the same rows, forms dZ = a ⊙ (g − Σ a g), applies the
// horizontal adjoint into a rolling 4-column register window per token (deterministic, no
// atomics), streams the row partials out, and a second kernel applies the vertical adjoint.
#include <algorithm>

#include "skp_common.h"

using namespace skp;

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / WAVE;

// ------------------------------------------------------------------------------------ fwd
// Lanes own token quads (4 consecutive tokens): V reads are ds_read_b128 and each pixel row
// of attn leaves as 1 KiB float4 wave stores.  NQ = quads per lane (N <= 256*NQ).
template <int NQ, bool VEC, bool NTS = false>
__global__ __launch_bounds__(kThreads) void capture_fwd_kernel(const float* __restrict__ z, int BH, int s, int N,
                                                               int R, float* __restrict__ attn,
                                                               float2* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) float V[];
  constexpr int Np = NQ * 4 * WAVE;
  // block -> (b, y) with b fastest: consecutive blocks (one per XCD under round-robin
  // dispatch) take different heads, so each XCD's L2 keeps the z_low of the heads it serves.
  const int b = blockIdx.x % BH;
  const int y = blockIdx.x / BH;
  const Taps4 ty = bicubic_taps(y, s, R);
  const float* zb = z + (size_t)b * s * s * N;
  if (VEC) {
    float4* V4 = reinterpret_cast<float4*>(V);
    const float4* r0 = reinterpret_cast<const float4*>(zb + (size_t)ty.i[0] * s * N);
    const float4* r1 = reinterpret_cast<const float4*>(zb + (size_t)ty.i[1] * s * N);
    const float4* r2 = reinterpret_cast<const float4*>(zb + (size_t)ty.i[2] * s * N);
    const float4* r3 = reinterpret_cast<const float4*>(zb + (size_t)ty.i[3] * s * N);
    const int nq = N / 4, Nq = N / 4, Npq = Np / 4;
    for (int e = threadIdx.x; e < s * Npq; e += kThreads) {
      const int j = e / Npq, q = e - j * Npq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < nq) {
        const size_t o = (size_t)j * Nq + q;
        const float4 a0 = r0[o], a1 = r1[o], a2 = r2[o], a3 = r3[o];
        v.x = ty.w[0] * a0.x + ty.w[1] * a1.x + ty.w[2] * a2.x + ty.w[3] * a3.x;
        v.y = ty.w[0] * a0.y + ty.w[1] * a1.y + ty.w[2] * a2.y + ty.w[3] * a3.y;
        v.z = ty.w[0] * a0.z + ty.w[1] * a1.z + ty.w[2] * a2.z + ty.w[3] * a3.z;
        v.w = ty.w[0] * a0.w + ty.w[1] * a1.w + ty.w[2] * a2.w + ty.w[3] * a3.w;
      }
      V4[e] = v;
    }
  } else {
    for (int e = threadIdx.x; e < s * Np; e += kThreads) {
      const int j = e / Np, n = e - j * Np;
      float v = 0.0f;
      if (n < N) {
        v = ty.w[0] * zb[(size_t)(ty.i[0] * s + j) * N + n];
        v += ty.w[1] * zb[(size_t)(ty.i[1] * s + j) * N + n];
        v += ty.w[2] * zb[(size_t)(ty.i[2] * s + j) * N + n];
        v += ty.w[3] * zb[(size_t)(ty.i[3] * s + j) * N + n];
      }
      V[e] = v;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float4* V4 = reinterpret_cast<const float4*>(V);
  constexpr int Npq = Np / 4;
  float* orow = attn + ((size_t)b * R * R + (size_t)y * R) * N;
  for (int x = wid; x < R; x += kWaves) {
    const Taps4 tx = bicubic_taps(x, s, R);
    float4 zc[NQ];
    float m = -INFINITY;
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      const int q = c * WAVE + lane;
      const float4 a0 = V4[tx.i[0] * Npq + q], a1 = V4[tx.i[1] * Npq + q];
      const float4 a2 = V4[tx.i[2] * Npq + q], a3 = V4[tx.i[3] * Npq + q];
      float4 v;
      v.x = tx.w[0] * a0.x + tx.w[1] * a1.x + tx.w[2] * a2.x + tx.w[3] * a3.x;
      v.y = tx.w[0] * a0.y + tx.w[1] * a1.y + tx.w[2] * a2.y + tx.w[3] * a3.y;
      v.z = tx.w[0] * a0.z + tx.w[1] * a1.z + tx.w[2] * a2.z + tx.w[3] * a3.z;
      v.w = tx.w[0] * a0.w + tx.w[1] * a1.w + tx.w[2] * a2.w + tx.w[3] * a3.w;
      const int n = 4 * q;
      v.x = n < N ? v.x : -INFINITY;
      v.y = n + 1 < N ? v.y : -INFINITY;
      v.z = n + 2 < N ? v.z : -INFINITY;
      v.w = n + 3 < N ? v.w : -INFINITY;
      zc[c] = v;
      m = fmaxf(m, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
    m = wave_max(m);
    float ssum = 0.0f;
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      zc[c].x = __expf(zc[c].x - m);
      zc[c].y = __expf(zc[c].y - m);
      zc[c].z = __expf(zc[c].z - m);
      zc[c].w = __expf(zc[c].w - m);
      ssum += (zc[c].x + zc[c].y) + (zc[c].z + zc[c].w);
    }
    ssum = wave_sum(ssum);
    const float inv = 1.0f / ssum;
    if (stats && lane == 0) stats[((size_t)b * R + y) * R + x] = make_float2(m, inv);   // row max, 1/Σ
    float* o = orow + (size_t)x * N;
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      const int n = 4 * (c * WAVE + lane);
      const float4 v = make_float4(zc[c].x * inv, zc[c].y * inv, zc[c].z * inv, zc[c].w * inv);
      if (VEC) {
        if (n < N) {
          if (NTS) {   // attn is read once, by the aggregate: stream it past the caches
            typedef float f4v __attribute__((ext_vector_type(4)));
            f4v w = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(o + n));
          } else {
            *reinterpret_cast<float4*>(o + n) = v;
          }
        }
      } else {
        if (n < N) o[n] = v.x;
        if (n + 1 < N) o[n + 1] = v.y;
        if (n + 2 < N) o[n + 2] = v.z;
        if (n + 3 < N) o[n + 3] = v.w;
      }
    }
  }
}

// ------------------------------------------------------------------------------------ bwd
// Phase A: one 512-thread block per (b, y).  Chunks of CH output pixels:
//   (1) stage g for the chunk in LDS (float4 loads prefetched one chunk ahead when the
//       gradient is token-major), scaled by gscale,
//   (2) one wave per pixel recomputes the softmax row a and overwrites g with
//       dZ = a ⊙ (g − Σ a g),
//   (3) thread t owns tokens t, t+512, …: walking the pixels in order it applies the
//       horizontal bicubic adjoint into a 4-register window over the low-res columns
//       lo(x) … lo(x)+3 (lo = first tap before clamping).  lo never decreases along x, so
//       when it advances the window's lowest column is complete and leaves as one coalesced
//       store of the row partial ws[b][y][j][:]; the virtual columns −2, −1 and s, s+1 fold
//       into 0 and s−1 exactly as torch's clamped taps do.  Each value has one owner thread
//       and a fixed order: deterministic, no atomics, no LDS accumulator.
// LDS = V (s × Np) + G (CH × (Np+1)) + tap tables, so two or three blocks share a CU.
constexpr int kBwdThreads = 512;
constexpr int kBwdWaves = kBwdThreads / WAVE;

template <int NT>
struct RowPartialWriter {   // streams finished low-res columns of one (b, y) row partial
  float* wrow;
  int N, s, pt;
  float pend[NT];
  __device__ __forceinline__ void store(int col, const float* v) const {
#pragma unroll
    for (int r = 0; r < NT; ++r) {
      const int n = r * kBwdThreads + threadIdx.x;
      if (n < N) wrow[(size_t)col * N + n] = v[r];
    }
  }
  __device__ __forceinline__ void store_zero(int col) const {
    const float z[NT] = {};
    store(col, z);
  }
  // column c (virtual, −2 … s+1) is complete with value v
  __device__ __forceinline__ void emit(int c, const float* v) {
    const int t = min(max(c, 0), s - 1);
    if (t != pt) {   // block-uniform
      store(pt, pend);
      for (int j = pt + 1; j < t; ++j) store_zero(j);
      pt = t;
#pragma unroll
      for (int r = 0; r < NT; ++r) pend[r] = v[r];
    } else {
#pragma unroll
      for (int r = 0; r < NT; ++r) pend[r] += v[r];
    }
  }
  __device__ __forceinline__ void finish() {
    store(pt, pend);
    for (int j = pt + 1; j < s; ++j) store_zero(j);
  }
};

template <int NT>
__global__ __launch_bounds__(kBwdThreads) void capture_bwd_rows_kernel(const float* __restrict__ z, int BH, int s,
                                                                       int N, int R, int CH,
                                                                       const float* __restrict__ g, int group,
                                                                       long long sb, long long sp, long long sn,
                                                                       float gscale, int share,
                                                                       const float2* __restrict__ stats,
                                                                       float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int Np = NT * kBwdThreads;
  constexpr int Gp = Np + 4;        // G rows 16-B aligned (float4 token quads) and bank-skewed
  constexpr int Npq = Np / 4;
  constexpr int NQB = Npq / WAVE;   // token quads per lane in the per-pixel pass
  float* V = lds;                                   // s × Np   vertical bicubic pass of z_low for row y
  float* TW = V + s * Np;                           // R × 4    tap weights (16-B aligned: Np % 4 == 0)
  int* TL = reinterpret_cast<int*>(TW + R * 4);     // R        first tap column before clamping
  float* G = TW + R * 4 + ((R + 3) & ~3);           // CH × Gp  g, then dZ, of the current pixel chunk
  // block -> (b, y).  When `share` consecutive heads read the same gradient rows (the heads of
  // one image: group > 1, or a broadcast g), the heads of one (image, y) go to the same XCD back
  // to back (workgroups are dispatched round-robin over the 8 XCDs), so that XCD's L2 fetches
  // the g row once instead of once per head.
  int b, y;
  if (share > 1 && (R & 7) == 0 && BH % share == 0) {
    const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
    const int h = k % share, rest = k / share, R8 = R >> 3;
    y = (rest % R8) * 8 + xcd;
    b = (rest / R8) * share + h;
  } else {
    b = blockIdx.x % BH;
    y = blockIdx.x / BH;
  }
  const Taps4 ty = bicubic_taps(y, s, R);
  const float* zb = z + (size_t)b * s * s * N;
  for (int x = threadIdx.x; x < R; x += kBwdThreads) {
    const Taps4 tx = bicubic_taps(x, s, R);
    *reinterpret_cast<float4*>(TW + 4 * x) = make_float4(tx.w[0], tx.w[1], tx.w[2], tx.w[3]);
    TL[x] = tx.lo;
  }
  // vertical pass (float4 along tokens when the layout allows)
  if ((N & 3) == 0 && (reinterpret_cast<uintptr_t>(zb) & 15) == 0) {
    const int nq = N / 4;
    constexpr int Npq = Np / 4;
    const float4* r0 = reinterpret_cast<const float4*>(zb + (size_t)ty.i[0] * s * N);
    const float4* r1 = reinterpret_cast<const float4*>(zb + (size_t)ty.i[1] * s * N);
    const float4* r2 = reinterpret_cast<const float4*>(zb + (size_t)ty.i[2] * s * N);
    const float4* r3 = reinterpret_cast<const float4*>(zb + (size_t)ty.i[3] * s * N);
    float4* V4 = reinterpret_cast<float4*>(V);
    for (int e = threadIdx.x; e < s * Npq; e += kBwdThreads) {
      const int j = e / Npq, q = e - j * Npq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < nq) {
        const size_t o = (size_t)j * nq + q;
        const float4 a0 = r0[o], a1 = r1[o], a2 = r2[o], a3 = r3[o];
        v.x = ty.w[0] * a0.x + ty.w[1] * a1.x + ty.w[2] * a2.x + ty.w[3] * a3.x;
        v.y = ty.w[0] * a0.y + ty.w[1] * a1.y + ty.w[2] * a2.y + ty.w[3] * a3.y;
        v.z = ty.w[0] * a0.z + ty.w[1] * a1.z + ty.w[2] * a2.z + ty.w[3] * a3.z;
        v.w = ty.w[0] * a0.w + ty.w[1] * a1.w + ty.w[2] * a2.w + ty.w[3] * a3.w;
      }
      V4[e] = v;
    }
  } else {
    for (int e = threadIdx.x; e < s * Np; e += kBwdThreads) {
      const int j = e / Np, n = e - j * Np;
      float v = 0.0f;
      if (n < N) {
        v = ty.w[0] * zb[(size_t)(ty.i[0] * s + j) * N + n];
        v += ty.w[1] * zb[(size_t)(ty.i[1] * s + j) * N + n];
        v += ty.w[2] * zb[(size_t)(ty.i[2] * s + j) * N + n];
        v += ty.w[3] * zb[(size_t)(ty.i[3] * s + j) * N + n];
      }
      V[e] = v;
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float* gb = g + (long long)(b / group) * sb + (long long)y * R * sp;
  // token-major broadcast gradient (sp == 1, e.g. the collect_maps backward): float4 over pixels,
  // prefetched into registers one chunk ahead so the loads overlap the chunk's compute.
  const bool g4 = (sn != 1) && (sp == 1) && (sn % 4 == 0) && (CH % 4 == 0) && (R % CH == 0) &&
                  ((reinterpret_cast<uintptr_t>(gb) & 15) == 0) && (CH * Np / 4) <= 4 * kBwdThreads;
  constexpr int kPre = 4;   // float4 per thread per chunk (CH*Np/4 <= 4*kBwdThreads)
  float4 pre[kPre];
  auto prefetch = [&](int x0) {
    const int qx = CH / 4;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int e = threadIdx.x + k * kBwdThreads;
      const int n = e / qx, xq = e - n * qx;
      pre[k] = (e < qx * Np && n < N && x0 < R)
                   ? *reinterpret_cast<const float4*>(gb + (long long)n * sn + x0 + 4 * xq)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  if (g4) prefetch(0);
  RowPartialWriter<NT> out;
  out.wrow = ws + ((size_t)b * R + y) * (size_t)s * N;   // ws layout (BH, R, s, N)
  out.N = N;
  out.s = s;
  out.pt = 0;
  float acc[4][NT];
#pragma unroll
  for (int r = 0; r < NT; ++r) {
    out.pend[r] = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k][r] = 0.0f;
  }
  int base = -2;   // virtual column held by acc[0]
  for (int x0 = 0; x0 < R; x0 += CH) {
    __syncthreads();  // previous chunk's G consumed (and tables/V ready on the first pass)
    const int nx = min(CH, R - x0);
    if (g4) {
      const int qx = CH / 4;
#pragma unroll
      for (int k = 0; k < kPre; ++k) {
        const int e = threadIdx.x + k * kBwdThreads;
        if (e < qx * Np) {
          const int n = e / qx, xq = e - n * qx;
          G[(4 * xq + 0) * Gp + n] = pre[k].x * gscale;
          G[(4 * xq + 1) * Gp + n] = pre[k].y * gscale;
          G[(4 * xq + 2) * Gp + n] = pre[k].z * gscale;
          G[(4 * xq + 3) * Gp + n] = pre[k].w * gscale;
        }
      }
      prefetch(x0 + CH);   // next chunk's loads fly while this chunk computes
    } else if (sn == 1) {
      for (int e = threadIdx.x; e < CH * Np; e += kBwdThreads) {
        const int xx = e / Np, n = e - xx * Np;
        G[xx * Gp + n] = (n < N && xx < nx) ? gb[(long long)(x0 + xx) * sp + n] * gscale : 0.0f;
      }
    } else {
      for (int e = threadIdx.x; e < CH * Np; e += kBwdThreads) {
        const int n = e / CH, xx = e - n * CH;
        G[xx * Gp + n] = (n < N && xx < nx) ? gb[(long long)(x0 + xx) * sp + (long long)n * sn] * gscale : 0.0f;
      }
    }
    __syncthreads();
    // one wave per pixel, lanes own token quads (ds_read_b128 of V and G): recompute the
    // softmax row a (with the forward's row max and 1/Σ when `stats` is given, else by two
    // wave reductions), then dZ = a ⊙ (g − Σ a g) over g in place
    const float4* V4 = reinterpret_cast<const float4*>(V);
    for (int xx = wid; xx < nx; xx += kBwdWaves) {
      const int x = x0 + xx;
      const int lo = TL[x];
      const int i0 = max(lo, 0), i1 = min(max(lo + 1, 0), s - 1);
      const int i2 = min(lo + 2, s - 1), i3 = min(lo + 3, s - 1);
      const float4 w = *reinterpret_cast<const float4*>(TW + 4 * x);
      float4 a[NQB];
#pragma unroll
      for (int c = 0; c < NQB; ++c) {
        const int q = c * WAVE + lane;
        const float4 a0 = V4[i0 * Npq + q], a1 = V4[i1 * Npq + q];
        const float4 a2 = V4[i2 * Npq + q], a3 = V4[i3 * Npq + q];
        a[c].x = w.x * a0.x + w.y * a1.x + w.z * a2.x + w.w * a3.x;
        a[c].y = w.x * a0.y + w.y * a1.y + w.z * a2.y + w.w * a3.y;
        a[c].z = w.x * a0.z + w.y * a1.z + w.z * a2.z + w.w * a3.z;
        a[c].w = w.x * a0.w + w.y * a1.w + w.z * a2.w + w.w * a3.w;
      }
      float m, inv;
      if (stats) {
        const float2 st = stats[((size_t)b * R + y) * R + x];
        m = st.x;
        inv = st.y;
      } else {
        m = -INFINITY;
#pragma unroll
        for (int c = 0; c < NQB; ++c) {
          const int n = 4 * (c * WAVE + lane);
          if (n < N) m = fmaxf(m, a[c].x);
          if (n + 1 < N) m = fmaxf(m, a[c].y);
          if (n + 2 < N) m = fmaxf(m, a[c].z);
          if (n + 3 < N) m = fmaxf(m, a[c].w);
        }
        m = wave_max(m);
      }
      float ssum = 0.0f;
#pragma unroll
      for (int c = 0; c < NQB; ++c) {
        const int n = 4 * (c * WAVE + lane);
        a[c].x = n < N ? __expf(a[c].x - m) : 0.0f;
        a[c].y = n + 1 < N ? __expf(a[c].y - m) : 0.0f;
        a[c].z = n + 2 < N ? __expf(a[c].z - m) : 0.0f;
        a[c].w = n + 3 < N ? __expf(a[c].w - m) : 0.0f;
        ssum += (a[c].x + a[c].y) + (a[c].z + a[c].w);
      }
      if (!stats) inv = 1.0f / wave_sum(ssum);
      float4* Gx = reinterpret_cast<float4*>(G + xx * Gp);
      float dot = 0.0f;
#pragma unroll
      for (int c = 0; c < NQB; ++c) {
        a[c].x *= inv;
        a[c].y *= inv;
        a[c].z *= inv;
        a[c].w *= inv;
        const float4 g = Gx[c * WAVE + lane];
        dot += a[c].x * g.x + a[c].y * g.y + a[c].z * g.z + a[c].w * g.w;
      }
      dot = wave_sum(dot);
#pragma unroll
      for (int c = 0; c < NQB; ++c) {
        const int q = c * WAVE + lane;
        const float4 g = Gx[q];
        Gx[q] = make_float4(a[c].x * (g.x - dot), a[c].y * (g.y - dot), a[c].z * (g.z - dot), a[c].w * (g.w - dot));
      }
    }
    __syncthreads();
    // horizontal adjoint of the chunk into the rolling 4-column window
    for (int xx = 0; xx < nx; ++xx) {
      const int x = x0 + xx;
      const int lo = TL[x];
      while (base < lo) {   // block-uniform: column `base` is complete
        out.emit(base, acc[0]);
#pragma unroll
        for (int r = 0; r < NT; ++r) {
          acc[0][r] = acc[1][r];
          acc[1][r] = acc[2][r];
          acc[2][r] = acc[3][r];
          acc[3][r] = 0.0f;
        }
        ++base;
      }
      const float4 w = *reinterpret_cast<const float4*>(TW + 4 * x);
#pragma unroll
      for (int r = 0; r < NT; ++r) {
        const float gv = G[xx * Gp + r * kBwdThreads + threadIdx.x];
        acc[0][r] += w.x * gv;
        acc[1][r] += w.y * gv;
        acc[2][r] += w.z * gv;
        acc[3][r] += w.w * gv;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) out.emit(base + k, acc[k]);
  out.finish();
}

// Phase B: dz[b][i·s + j][n] = Σ_y wy(y→i) · ws[b][y][j][n].  Thread = one (j, n) element of one
// b; it streams the R row partials in order (each read exactly once, coalesced across the
// block) through the same rolling 4-row window as the horizontal adjoint: low-res row i is
// complete once lo(y) passes it and leaves as one coalesced store (edge rows folded as torch's
// clamped taps do).  Deterministic, no atomics.
constexpr int kColThreads = 256;
constexpr int kColBatch = 8;   // row partials loaded ahead per thread
__global__ __launch_bounds__(kColThreads) void capture_bwd_cols_kernel(const float* __restrict__ ws, int BH, int s,
                                                                       int N, int R, float* __restrict__ dz) {
  __shared__ __attribute__((aligned(16))) float TW[1024 * 4];
  __shared__ int TL[1024];
  const int b = blockIdx.y;
  const long long plane = (long long)s * N;
  const long long e = (long long)blockIdx.x * kColThreads + threadIdx.x;
  for (int y = threadIdx.x; y < R; y += kColThreads) {
    const Taps4 ty = bicubic_taps(y, s, R);
    *reinterpret_cast<float4*>(TW + 4 * y) = make_float4(ty.w[0], ty.w[1], ty.w[2], ty.w[3]);
    TL[y] = ty.lo;
  }
  __syncthreads();
  if (e >= plane) return;
  const float* src = ws + (size_t)b * R * plane + e;
  float* out = dz + (size_t)b * s * plane + e;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, pend = 0.f;
  int base = -2, pt = 0;
  auto emit = [&](int c, float v) {   // virtual low-res row c (−2 … s+1) is complete
    const int t = min(max(c, 0), s - 1);
    if (t != pt) {
      out[(size_t)pt * plane] = pend;
      for (int j = pt + 1; j < t; ++j) out[(size_t)j * plane] = 0.0f;
      pt = t;
      pend = v;
    } else {
      pend += v;
    }
  };
  for (int y0 = 0; y0 < R; y0 += kColBatch) {
    float v[kColBatch];
#pragma unroll
    for (int u = 0; u < kColBatch; ++u) v[u] = (y0 + u < R) ? src[(size_t)(y0 + u) * plane] : 0.0f;
#pragma unroll
    for (int u = 0; u < kColBatch; ++u) {
      const int y = y0 + u;
      if (y < R) {
        const int lo = TL[y];
        while (base < lo) {   // uniform across the block
          emit(base, a0);
          a0 = a1; a1 = a2; a2 = a3; a3 = 0.0f;
          ++base;
        }
        const float4 w = *reinterpret_cast<const float4*>(TW + 4 * y);
        a0 += w.x * v[u];
        a1 += w.y * v[u];
        a2 += w.z * v[u];
        a3 += w.w * v[u];
      }
    }
  }
  emit(base, a0);
  emit(base + 1, a1);
  emit(base + 2, a2);
  emit(base + 3, a3);
  out[(size_t)pt * plane] = pend;
  for (int j = pt + 1; j < s; ++j) out[(size_t)j * plane] = 0.0f;
}

// ------------------------------------------------------------------------------------ fused fwd
// Capture + per-image aggregate in one pass (ptp_utils.py:508-538 for every captured layer,
// then optimize.py:27-79's mean over layers and heads, per image):
//   maps[b][n][p] = (1/(L·H)) Σ_l Σ_h softmax_n(bicubic_{s_l→R}(z_l[b·H+h])[p])[n]
// No (B·H, R², N) attention reaches HBM: HBM sees the z_low reads, the maps write and the
// per-pixel (max, 1/Σ) stats the backward reuses.
//
// One workgroup (WAVES waves) owns P consecutive pixels of output row y of image b and loops
// over every (layer, head).  Per (l, h): the vertical bicubic pass of the chunk's low-res
// columns into LDS (V, nc × Np, tokens padded with −1e30 so they exp to 0 with no masking),
// then each 16-lane row of a wave takes one pixel (lanes own QPL token quads): horizontal taps
// from V (ds_read_b128; the four rows' quads fall in disjoint banks), max and Σ by four
// single-instruction DPP steps inside the row, and acc += exp(z − m)·(1/Σ) in registers on
// the packed f32 VALU.  A wave owns PXW pixels, four at a time, so acc is PXW/4 × QPL float4 per
// lane.  After the last (l, h) the (pixel, token) accumulators go token-major through an LDS
// tile, 128 tokens per round, as coalesced runs of P pixels.
// Blocks are mapped XCD-major: block k runs on XCD k % 8 and takes job (k % 8)·⌈jobs/8⌉ + k / 8,
// so each XCD walks consecutive rows of one image and its L2 serves their shared z_low rows.
constexpr float kPadLogit = -1e30f;   // Σ taps ≈ 1, so padded tokens interpolate to ≈ −1e30
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

// a wave-uniform pointer held in SGPRs: keeps the compiler from re-associating it with lane offsets
// into per-lane 64-bit address arithmetic (global loads then take the saddr + 32-bit voffset form)
// (global address space, so the loads stay global_load rather than flat_load)
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* uniform_ptr(T* p) {
  const unsigned long long u = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return (__attribute__((address_space(1))) T*)(((unsigned long long)hi << 32) | lo);
}

struct CapLayers {
  const float* z[SKP_MAX_LAYERS];
  float2* stats[SKP_MAX_LAYERS];
  int s[SKP_MAX_LAYERS];
  float sc[SKP_MAX_LAYERS];   // (float)s / (float)R, the bicubic scale (no division on the device)
};

// max / sum over each 16-lane row: four DPP steps, each one VALU op with the DPP source
// (no mov + canonicalise); `s_nop 1` covers the VALU-write -> DPP-read hazard of the chain.
__device__ __forceinline__ float row16_max(float v) {
  asm volatile(
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf"
      : "+v"(v));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  asm volatile(
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf"
      : "+v"(v));
  return v;
}

// pixels per wave (a multiple of 4): acc = PXW/4 · QPL float4 = 32 VGPRs where possible
constexpr int maps_pxw(int qpl) { return (32 / qpl) < 4 ? 4 : ((32 / qpl) > 16 ? 16 : 32 / qpl); }

#ifndef SKP_MAPS_PRIO
#define SKP_MAPS_PRIO 1   // s_setprio level of the staging phase (0: off; 1, 2, 3 measured 972, 983, 982 vs 1003 us)
#endif
#ifndef SKP_MAPS_PROBE
// timing probes (A/B builds via tools/build_variant.sh only; r06: staging alone 417 µs, pixels
// alone 605 µs, both 900 µs at the bench shape, profiles/r06s_maps_fwd_probes.txt): 1 = the
// staging without its z_low loads, 2 = no pixel work
#define SKP_MAPS_PROBE 0
#endif
#ifndef SKP_MAPS_NT
// 1: the maps and stats leave with non-temporal stores, so the 296 MB write stream does not evict
// the z_low rows the XCD's other workgroups are about to read: 975 vs 994 µs, FETCH_SIZE 823 vs
// 1002 MB at the bench shape (profiles/r03ae_maps_nt_ab.txt); 0 = plain stores (A/B build)
#define SKP_MAPS_NT 1
#endif
#if SKP_MAPS_NT
#define SKP_MAPS_ST(dst, v) __builtin_nontemporal_store((v), &(dst))
#else
#define SKP_MAPS_ST(dst, v) ((dst) = (v))
#endif
template <int QPL, int WAVES>
__global__ __launch_bounds__(WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(4)))
void capture_maps_kernel(CapLayers cl, int L, int B, int H, int N, int R, int nchunks, int vstride, float count,
                         float* __restrict__ maps) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kMapThreads = WAVES * WAVE;
  constexpr int PXW = maps_pxw(QPL);
  constexpr int G = PXW / 4;                 // pixel quadruples per wave
  constexpr int P = WAVES * PXW;             // pixels per workgroup
  constexpr int Np = 64 * QPL;               // padded tokens (16 lanes × QPL quads)
  constexpr int Npq = Np / 4;
  constexpr float L2E = 1.4426950408889634f;
  float4* TW = reinterpret_cast<float4*>(lds);             // [2][P] tap weights (by layer parity)
  int4* TI = reinterpret_cast<int4*>(lds + 8 * P);          // [2][P] tap offsets (column − c0) · Npq
  float* V = lds + 16 * P;                                  // [2][vstride] vertical passes (then the store tile)

  const int total = B * R * nchunks;
  const int per = (total + 7) / 8;
  // XCD x takes jobs [x·per, (x + 1)·per); its workgroups stride through them (one job each on a
  // full grid; with a persistent grid of 2 workgroups per CU the XCD's workgroups start together
  // and walk the same (layer, head) slabs in step, so the rows they share stay in that XCD's L2)
  const int xcd = blockIdx.x & 7, nper = gridDim.x >> 3;
  const int jfirst = xcd * per + (blockIdx.x >> 3), jend = min(total, (xcd + 1) * per);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row = lane >> 4, li = lane & 15;
  for (int job = jfirst; job < jend; job += nper) {
    if (job != jfirst) __syncthreads();   // the previous job's store tile (in V) fully read
    const int xc = job % nchunks;
    const int y = (job / nchunks) % R;
    const int b = job / (nchunks * R);
    const int x0 = xc * P;
    const int np = min(P, R - x0);

    f4 acc[G][QPL];
  #pragma unroll
    for (int g = 0; g < G; ++g)
  #pragma unroll
      for (int c = 0; c < QPL; ++c) acc[g][c] = (f4)0.0f;

    const bool vec = (N & 3) == 0;
    // Per layer: the uniform setup (columns, vertical taps, the tap table) once; per (layer, head)
    // slab: the vertical pass, then the pixel work; two workgroups per CU overlap one's staging
    // with the other's pixels.  (A software pipeline with double-buffered V measured slower: 1.03
    // vs 0.94 ms.)  r05: the layer's setup hoisted out of the head loop into scalar registers and
    // the z_low rows addressed as uniform bases + 32-bit lane offsets (it had been ≈ 90 VALU per
    // slab of 64-bit address and tap arithmetic recomputed per head).
    const unsigned nq = N >> 2;
    for (int l = 0; l < L; ++l) {
      const int s = cl.s[l];
      const float sc = cl.sc[l];
      const int c0 = max(bicubic_taps_s(x0, s, sc).lo, 0);
      const int nc = min(bicubic_taps_s(x0 + np - 1, s, sc).lo + 3, s - 1) - c0 + 1;
      const Taps4 tyv = bicubic_taps_s(y, s, sc);
      // uniform values: force them into SGPRs for the head loop
      float wy[4];
      unsigned ro[4];   // float offsets of the 4 tap rows' first column (c0) inside one (b, h) slab
  #pragma unroll
      for (int k = 0; k < 4; ++k) {
        wy[k] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, tyv.w[k])));
        ro[k] = (unsigned)__builtin_amdgcn_readfirstlane((tyv.i[k] * s + c0) * N);
      }
      const int tot = __builtin_amdgcn_readfirstlane(nc * Npq);
      {   // tap table of this layer (buffer l & 1: layer l − 1's readers may still run)
        float4* tw = TW + (l & 1) * P;
        int4* tiw = TI + (l & 1) * P;
        for (int x = tid; x < P; x += kMapThreads) {
          const Taps4 t = bicubic_taps_s(x0 + min(x, np - 1), s, sc);
          tw[x] = make_float4(t.w[0], t.w[1], t.w[2], t.w[3]);
          tiw[x] = make_int4((t.i[0] - c0) * Npq, (t.i[1] - c0) * Npq, (t.i[2] - c0) * Npq, (t.i[3] - c0) * Npq);
        }
      }
      const float4* tw = TW + (l & 1) * P;
      const int4* tiw = TI + (l & 1) * P;
      for (int h = 0; h < H; ++h) {
        const int it = l * H + h;
        const int bh = b * H + h;
        // the lane-derived offsets are recomputed per slab from an opaque copy of the thread index
        // (hoisted out of the head loop they held VGPRs across it: 898–901 vs 909–911 µs, r06s)
        int tl = tid;
        asm volatile("" : "+v"(tl));
        const int lanel = tl & 63, widl = tl >> 6, rowl = lanel >> 4, lil = lanel & 15;
  #if SKP_MAPS_PRIO
        __builtin_amdgcn_s_setprio(SKP_MAPS_PRIO);   // the staging's loads ahead of the other workgroup's pixels
  #endif
        // V and the tap table are double-buffered: slab it writes the buffers slab it − 2 read, and
        // every thread finished those reads before the previous slab's post-staging barrier
        float* Vb = V + (it & 1) * vstride;
        const float* zb = cl.z[l] + (size_t)bh * s * s * N;
        if (vec) {
          // V[jj][n] = Σ_k wy_k · z[iy_k][c0 + jj][n]: thread element e = tl + k·threads, lane
          // offset o = jj·nq + q (a 32-bit offset from each uniform rowl base)
          const auto* r0 = uniform_ptr(reinterpret_cast<const f4*>(zb + ro[0]));
          const auto* r1 = uniform_ptr(reinterpret_cast<const f4*>(zb + ro[1]));
          const auto* r2 = uniform_ptr(reinterpret_cast<const f4*>(zb + ro[2]));
          const auto* r3 = uniform_ptr(reinterpret_cast<const f4*>(zb + ro[3]));
          f4* V4 = reinterpret_cast<f4*>(Vb);
          constexpr unsigned JS = kMapThreads / Npq;   // columns per thread step (4 at 8 waves, QPL 8)
          static_assert(kMapThreads % Npq == 0, "thread step must cover whole columns");
          const unsigned q = (unsigned)tl % Npq;
          unsigned ob = (((unsigned)tl / Npq) * nq + q) * 16u;   // byte offset (saddr + 32-bit voffset loads)
          const unsigned obs = JS * nq * 16u;
          using gcf4 = const __attribute__((address_space(1))) f4;
          using gcc = const __attribute__((address_space(1))) char;
#ifndef SKP_MAPS_VPT
#define SKP_MAPS_VPT 1   // elements per thread whose loads are in flight together (A/B build)
#endif
          constexpr int VPT = SKP_MAPS_VPT;
  #pragma unroll 1
          for (int e0 = tl; e0 < tot; e0 += VPT * kMapThreads, ob += VPT * obs) {
            f4 a[VPT][4];
  #pragma unroll
            for (int k = 0; k < VPT; ++k) {
              if (e0 + k * kMapThreads < tot && q < nq && SKP_MAPS_PROBE != 1) {   // timing probe 1: no z_low loads
                const unsigned o = ob + k * obs;
                a[k][0] = *reinterpret_cast<gcf4*>(reinterpret_cast<gcc*>(r0) + o);
                a[k][1] = *reinterpret_cast<gcf4*>(reinterpret_cast<gcc*>(r1) + o);
                a[k][2] = *reinterpret_cast<gcf4*>(reinterpret_cast<gcc*>(r2) + o);
                a[k][3] = *reinterpret_cast<gcf4*>(reinterpret_cast<gcc*>(r3) + o);
              }
            }
  #pragma unroll
            for (int k = 0; k < VPT; ++k) {
              const int e = e0 + k * kMapThreads;
              if (e < tot) {
                f4 v = (f4)kPadLogit;
                if (SKP_MAPS_PROBE == 1) {
                  v = (f4)wy[0];
                } else if (q < nq) {
                  v = a[k][0] * wy[0];
                  v = __builtin_elementwise_fma(a[k][1], (f4)wy[1], v);
                  v = __builtin_elementwise_fma(a[k][2], (f4)wy[2], v);
                  v = __builtin_elementwise_fma(a[k][3], (f4)wy[3], v);
                }
                V4[e] = v;
              }
            }
          }
        } else {
  #pragma unroll 1
          for (int e = tl; e < nc * Np; e += kMapThreads) {
            const int jj = e / Np, n = e - jj * Np;
            float v = kPadLogit;
            if (n < N) {
              const int j = c0 + jj;
              v = wy[0] * zb[((size_t)tyv.i[0] * s + j) * N + n];
              v += wy[1] * zb[((size_t)tyv.i[1] * s + j) * N + n];
              v += wy[2] * zb[((size_t)tyv.i[2] * s + j) * N + n];
              v += wy[3] * zb[((size_t)tyv.i[3] * s + j) * N + n];
            }
            Vb[e] = v;
          }
        }
  #if SKP_MAPS_PRIO
        __builtin_amdgcn_s_setprio(0);
  #endif
        __syncthreads();
        const f4* V4 = reinterpret_cast<const f4*>(Vb) + lil;
        // this (head, rowl, chunk)'s stats run: a uniform base, lane offsets xl
        auto* st = cl.stats[l] ? uniform_ptr(reinterpret_cast<f2v*>(cl.stats[l]) + ((size_t)bh * R + y) * R + x0) : nullptr;
  #pragma unroll
        for (int g = 0; g < (SKP_MAPS_PROBE == 2 ? 0 : G); ++g) {   // timing probe 2: no pixel work
          const int xl = widl * PXW + 4 * g + rowl;              // pixel of this 16-lane rowl
          const int xr = min(xl, np - 1);                        // past-the-edge rows redo a valid one
          const float4 w = tw[xr];
          const int4 ti = tiw[xr];
          f4 zc[QPL];
          float m = kPadLogit;
  #pragma unroll
          for (int c = 0; c < QPL; ++c) {
            const f4 a0 = V4[ti.x + 16 * c], a1 = V4[ti.y + 16 * c];
            const f4 a2 = V4[ti.z + 16 * c], a3 = V4[ti.w + 16 * c];
            // token pairs on the packed f32 VALU: z = ((w0·a0 + w1·a1) + w2·a2) + w3·a3
            f4 v = a0 * w.x;
            v = __builtin_elementwise_fma(a1, (f4)w.y, v);
            v = __builtin_elementwise_fma(a2, (f4)w.z, v);
            v = __builtin_elementwise_fma(a3, (f4)w.w, v);
            zc[c] = v;
            m = __builtin_fmaxf(__builtin_fmaxf(m, v.x), v.y);
            m = __builtin_fmaxf(__builtin_fmaxf(m, v.z), v.w);
            if (QPL > 4 || (c & 1)) __builtin_amdgcn_sched_barrier(0);   // bound the LDS reads in flight (registers)
          }
          m = row16_max(m);
          const f4 mb = (f4)(-m * L2E);
          f4 sv = (f4)0.0f;
  #pragma unroll
          for (int c = 0; c < QPL; ++c) {
            f4 t = __builtin_elementwise_fma(zc[c], (f4)L2E, mb);
            t.x = __builtin_amdgcn_exp2f(t.x);
            t.y = __builtin_amdgcn_exp2f(t.y);
            t.z = __builtin_amdgcn_exp2f(t.z);
            t.w = __builtin_amdgcn_exp2f(t.w);
            zc[c] = t;
            sv += t;
          }
          const float inv = __builtin_amdgcn_rcpf(row16_sum((sv.x + sv.y) + (sv.z + sv.w)));
  #pragma unroll
          for (int c = 0; c < QPL; ++c) acc[g][c] = __builtin_elementwise_fma(zc[c], (f4)inv, acc[g][c]);
          if (st && lil == 0 && xl < np) {
            const f2v mi = {m, inv};
            SKP_MAPS_ST(st[(unsigned)xl], mi);
          }
          __builtin_amdgcn_sched_barrier(0);   // keep the next pixels' LDS reads from being hoisted (registers)
        }
      }
    }
    // token-major store: round r stages tokens [128r, 128r + 128) of all P pixels in LDS; lane li
    // of a row holds quads li + 16c, so round r takes c = 2r and 2r + 1
    constexpr int TS = 128 + 4;   // tile row stride (floats): 16-B aligned, b128 reads conflict-free
    float* tile = V;
    float* ob = maps + (size_t)b * N * R * R + (size_t)y * R + x0;
    const float rc = 1.0f / count;
  #pragma unroll
    for (int r = 0; r < (QPL + 1) / 2; ++r) {
      __syncthreads();
  #pragma unroll
      for (int g = 0; g < G; ++g) {
        const int xl = wid * PXW + 4 * g + row;
  #pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int c = 2 * r + h2;
          if (c < QPL) *reinterpret_cast<f4*>(tile + xl * TS + 4 * (li + 16 * h2)) = acc[g][c] * rc;
        }
      }
      __syncthreads();
      const int nr = min(128, Np - 128 * r) / 4;   // quads staged this round
      for (int e = tid; e < P * nr; e += kMapThreads) {
        const int xl = e % P, jq = e / P;
        if (xl >= np) continue;
        const f4 v = *reinterpret_cast<const f4*>(tile + xl * TS + 4 * jq);
        const int n = 128 * r + 4 * jq;
        if (n < N) SKP_MAPS_ST(ob[(size_t)n * R * R + xl], v.x);
        if (n + 1 < N) SKP_MAPS_ST(ob[(size_t)(n + 1) * R * R + xl], v.y);
        if (n + 2 < N) SKP_MAPS_ST(ob[(size_t)(n + 2) * R * R + xl], v.z);
        if (n + 3 < N) SKP_MAPS_ST(ob[(size_t)(n + 3) * R * R + xl], v.w);
      }
    }
  }
}

// ------------------------------------------------------------------------------------ fused bwd
// Backward of skp_capture_maps_fwd, one (layer, b·H + h, output row y) per WAVE, no LDS and no
// barriers.  The per-image map gradient is first transposed to pixel-major gT (B, R², N)
// (scaled by 1/(L·H)), so a pixel's token gradient is one coalesced 2-KiB run.  The wave walks
// the R pixels of its row left to right with lanes owning NQ token quads and keeps in registers
//   - the vertical bicubic pass of the 4 low-res columns lo(x) … lo(x)+3 the pixel taps (V
//     window; a new column = 4 coalesced z_low row reads when lo advances, every R/s pixels),
//   - the horizontal-adjoint accumulators of the same 4 virtual columns (W window).
// Per pixel: z = Σ_k wx_k V_k, a = exp(z − m)·(1/Σ) from the forward's stats, dot = Σ_n a g
// (one full-wave DPP reduction), dZ = a ⊙ (g − dot), W_k += wx_k dZ.  When lo advances the
// lowest W column is complete and leaves as one coalesced store of the row partial
// ws[bh][y][j][:] (virtual columns −2, −1 / s, s+1 fold into 0 / s−1 as torch's clamped taps
// do).  Each value has one owner lane and a fixed order: deterministic, no atomics.  The
// vertical adjoint is capture_bwd_cols_kernel over ws, as for skp_capture_bwd.
constexpr int kRowThreads = 256;

__device__ __forceinline__ float wave64_sum(float v) {
  v = row16_sum(v);
  float w = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(v), "+v"(w));
  v += w;
  w = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(v), "+v"(w));
  return v + w;
}
__device__ __forceinline__ float wave64_max(float v) {
  v = row16_max(v);
  float w = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(v), "+v"(w));
  v = __builtin_fmaxf(v, w);
  w = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(v), "+v"(w));
  return __builtin_fmaxf(v, w);
}

template <int NQ, bool STATS>
__global__ __launch_bounds__(kRowThreads) __attribute__((amdgpu_waves_per_eu(4)))
void capture_bwd_row_kernel(const float* __restrict__ z, int B, int H, int s, int N, int R,
                            const float* __restrict__ gT, const float2* __restrict__ stats, float* __restrict__ ws) {
  constexpr float L2E = 1.4426950408889634f;
  constexpr int W = kRowThreads / WAVE;
  constexpr int Np = 256 * NQ;                      // padded tokens (64 lanes × NQ quads)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float4* TWt = reinterpret_cast<float4*>(lds);                    // R tap weights (shared by the block)
  int* TLt = reinterpret_cast<int*>(lds + 4 * R);                  // R first taps (before clamping)
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  f4* ring = reinterpret_cast<f4*>(lds + 5 * R + ((4 - (5 * R) % 4) % 4)) + (size_t)wid * 4 * (Np / 4);   // 4 V columns
  for (int x = threadIdx.x; x < R; x += kRowThreads) {
    const Taps4 t = bicubic_taps(x, s, R);
    TWt[x] = make_float4(t.w[0], t.w[1], t.w[2], t.w[3]);
    TLt[x] = t.lo;
  }
  __syncthreads();
  // XCD-major job order: each XCD takes a contiguous range of (b, y, h), heads fastest, so the
  // H waves reading one gT row run back to back on one L2
  const long long total = (long long)B * H * R;
  const long long blocks = (total + W - 1) / W;
  const long long per = (blocks + 7) / 8;
  const long long jb = (long long)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const long long job = jb * W + wid;
  if (jb >= blocks || job >= total) return;
  const int h = (int)(job % H);
  const int y = (int)((job / H) % R);
  const int b = (int)(job / ((long long)H * R));
  const int bh = b * H + h;
  const int nq = N >> 2;
  const Taps4 ty = bicubic_taps(y, s, R);
  const f4* zr0 = reinterpret_cast<const f4*>(z + ((size_t)bh * s * s + (size_t)ty.i[0] * s) * N);
  const f4* zr1 = reinterpret_cast<const f4*>(z + ((size_t)bh * s * s + (size_t)ty.i[1] * s) * N);
  const f4* zr2 = reinterpret_cast<const f4*>(z + ((size_t)bh * s * s + (size_t)ty.i[2] * s) * N);
  const f4* zr3 = reinterpret_cast<const f4*>(z + ((size_t)bh * s * s + (size_t)ty.i[3] * s) * N);
  // lane quads lane + 64c; past-the-end quads read a valid quad (clamped)
  int qo[NQ];
  bool ok[NQ];
#pragma unroll
  for (int c = 0; c < NQ; ++c) {
    ok[c] = lane + 64 * c < nq;
    qo[c] = min(lane + 64 * c, nq - 1);
  }
  // vertical pass of virtual column j (clamped) into ring slot j & 3; padded quads get −1e30
  auto vcol = [&](int j) {
    const int o = min(max(j, 0), s - 1) * nq;
    f4* dst = ring + (j & 3) * (Np / 4) + lane;
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      f4 v = zr0[o + qo[c]] * ty.w[0];
      v = __builtin_elementwise_fma(zr1[o + qo[c]], (f4)ty.w[1], v);
      v = __builtin_elementwise_fma(zr2[o + qo[c]], (f4)ty.w[2], v);
      v = __builtin_elementwise_fma(zr3[o + qo[c]], (f4)ty.w[3], v);
      dst[64 * c] = ok[c] ? v : (f4)kPadLogit;
    }
  };
  const f4* grow = reinterpret_cast<const f4*>(gT + ((size_t)b * R * R + (size_t)y * R) * N);
  const float4* strow = STATS ? reinterpret_cast<const float4*>(stats + ((size_t)bh * R + y) * R) : nullptr;
  f4* wrow = reinterpret_cast<f4*>(ws + ((size_t)bh * R + y) * (size_t)s * N);

  // W window: adjoint accumulators of virtual columns base … base + 3 (registers).  lo advances
  // by at most one per pixel (s <= R) and stays <= s − 2, so in the loop a completed column is
  // either virtual (< 0: folded into the next slot, which clamps to the same column 0) or a real
  // column < s − 1 (stored once)
  f4 Ww[4][NQ];
  int base = TLt[0];
#pragma unroll
  for (int k = 0; k < 4; ++k) vcol(base + k);
#pragma unroll
  for (int c = 0; c < NQ; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) Ww[k][c] = (f4)0.0f;
  auto store_col = [&](int j, const f4* v) {
#pragma unroll
    for (int c = 0; c < NQ; ++c)
      if (ok[c]) wrow[(size_t)j * nq + lane + 64 * c] = v[c];
  };
  // Gradient rows ping-pong between two register sets (the pixel loop is unrolled by 2), so the
  // prefetch of pixel x + 1 needs no copy; with the forward's stats, 1/Σ folds into the exp's
  // offset (a = exp2(z·log2e − m·log2e + log2(1/Σ))), one v_log per pixel instead of NQ·2 v_pk_mul.
  f4 gA[NQ], gB[NQ];
#pragma unroll
  for (int c = 0; c < NQ; ++c) gA[c] = grow[qo[c]];
  float4 stq = make_float4(0.f, 0.f, 0.f, 0.f);   // stats of pixels x0 + 2·lane, x0 + 2·lane + 1
  auto rl = [](float v, int i) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), i)); };
  auto pixel = [&](int x, const f4 (&g)[NQ], f4 (&gn)[NQ]) {
    if (STATS && (x & 127) == 0) stq = strow[min((x >> 1) + lane, (R - 1) >> 1)];
    const float4 w = TWt[x];
    const int lo = TLt[x];
    if (base < lo) {   // wave-uniform: W slot 0 is complete; slide by one column
      if (base < 0) {
#pragma unroll
        for (int c = 0; c < NQ; ++c) Ww[1][c] += Ww[0][c];
      } else {
        store_col(base, Ww[0]);
      }
#pragma unroll
      for (int c = 0; c < NQ; ++c) {
        Ww[0][c] = Ww[1][c]; Ww[1][c] = Ww[2][c]; Ww[2][c] = Ww[3][c]; Ww[3][c] = (f4)0.0f;
      }
      ++base;
      vcol(base + 3);   // replaces the column that just left (ring slot (base − 1) & 3)
    }
    const int xn = min(x + 1, R - 1);
#pragma unroll
    for (int c = 0; c < NQ; ++c) gn[c] = grow[(size_t)xn * nq + qo[c]];
    const f4* v0 = ring + ((base + 0) & 3) * (Np / 4) + lane;
    const f4* v1 = ring + ((base + 1) & 3) * (Np / 4) + lane;
    const f4* v2 = ring + ((base + 2) & 3) * (Np / 4) + lane;
    const f4* v3 = ring + ((base + 3) & 3) * (Np / 4) + lane;
    f4 a[NQ];
    float m = -INFINITY;
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      f4 v = v0[64 * c] * w.x;
      v = __builtin_elementwise_fma(v1[64 * c], (f4)w.y, v);
      v = __builtin_elementwise_fma(v2[64 * c], (f4)w.z, v);
      v = __builtin_elementwise_fma(v3[64 * c], (f4)w.w, v);
      a[c] = v;
      if (!STATS) m = __builtin_fmaxf(__builtin_fmaxf(m, __builtin_fmaxf(v.x, v.y)), __builtin_fmaxf(v.z, v.w));
    }
    f4 mb;
    if (STATS) {
      const int src = (x & 127) >> 1;
      const bool odd = x & 1;
      m = rl(odd ? stq.z : stq.x, src);
      const float inv = rl(odd ? stq.w : stq.y, src);
      mb = (f4)(__builtin_amdgcn_logf(inv) - m * L2E);   // v_log_f32 is log2
    } else {
      m = wave64_max(m);   // padded quads hold −1e30: the max is unchanged
      mb = (f4)(-m * L2E);
    }
    f4 sv = (f4)0.0f;
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      f4 t = __builtin_elementwise_fma(a[c], (f4)L2E, mb);
      t.x = __builtin_amdgcn_exp2f(t.x);
      t.y = __builtin_amdgcn_exp2f(t.y);
      t.z = __builtin_amdgcn_exp2f(t.z);
      t.w = __builtin_amdgcn_exp2f(t.w);
      a[c] = t;
      if (!STATS) sv += t;
    }
    if (!STATS) {
      const float inv = __builtin_amdgcn_rcpf(wave64_sum((sv.x + sv.y) + (sv.z + sv.w)));
#pragma unroll
      for (int c = 0; c < NQ; ++c) a[c] *= inv;
    }
    f4 ag[NQ], dv = (f4)0.0f;
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      ag[c] = a[c] * g[c];
      dv += ag[c];
    }
    const float dot = wave64_sum((dv.x + dv.y) + (dv.z + dv.w));
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      const f4 dz = __builtin_elementwise_fma(a[c], (f4)(-dot), ag[c]);   // a ⊙ (g − dot)
      Ww[0][c] = __builtin_elementwise_fma(dz, (f4)w.x, Ww[0][c]);
      Ww[1][c] = __builtin_elementwise_fma(dz, (f4)w.y, Ww[1][c]);
      Ww[2][c] = __builtin_elementwise_fma(dz, (f4)w.z, Ww[2][c]);
      Ww[3][c] = __builtin_elementwise_fma(dz, (f4)w.w, Ww[3][c]);
    }
  };
  for (int x = 0; x < R; x += 2) {
    pixel(x, gA, gB);
    if (x + 1 < R) pixel(x + 1, gB, gA);
  }
  // the last window: virtual columns base … base + 3 (clamped runs summed, each column once)
  f4 acc[NQ];
#pragma unroll
  for (int c = 0; c < NQ; ++c) acc[c] = Ww[0][c];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const int tp = min(max(base + k - 1, 0), s - 1), t = min(max(base + k, 0), s - 1);
    if (t == tp) {
#pragma unroll
      for (int c = 0; c < NQ; ++c) acc[c] += Ww[k][c];
    } else {
      store_col(tp, acc);
#pragma unroll
      for (int c = 0; c < NQ; ++c) acc[c] = Ww[k][c];
    }
  }
  store_col(min(max(base + 3, 0), s - 1), acc);
}

size_t bwd_row_lds(int R, int nqpl) {   // tap table + 4 waves × 4 ring columns × Np floats
  return ((size_t)5 * R + 4 + (size_t)(kRowThreads / WAVE) * 4 * 256 * nqpl) * sizeof(float);
}

// float4 form of transpose_scale_kernel (P % 4 == 0 and N % 4 == 0, 16-B aligned): 16-B loads along
// p and 16-B stores along n, the 64 × 64 tile staying in LDS with a 65-float row pitch
// (bench shape: 97 vs 120 µs for the scalar form)
__global__ __launch_bounds__(256) void transpose_scale4_kernel(const float* __restrict__ g, int N, int P, float scale,
                                                               float* __restrict__ gT) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const float* gb = g + (size_t)b * N * P;
  float* ob = gT + (size_t)b * N * P;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int nl = e >> 4, pq = e & 15;
    const int n = n0 + nl, p = p0 + 4 * pq;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n < N && p < P) v = *reinterpret_cast<const float4*>(gb + (size_t)n * P + p);
    tile[nl][4 * pq] = v.x * scale;
    tile[nl][4 * pq + 1] = v.y * scale;
    tile[nl][4 * pq + 2] = v.z * scale;
    tile[nl][4 * pq + 3] = v.w * scale;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int pl = e >> 4, nq = e & 15;
    const int p = p0 + pl, n = n0 + 4 * nq;
    if (p < P && n < N)
      *reinterpret_cast<float4*>(ob + (size_t)p * N + n) =
          make_float4(tile[4 * nq][pl], tile[4 * nq + 1][pl], tile[4 * nq + 2][pl], tile[4 * nq + 3][pl]);
  }
}

// gT[b][p][n] = scale · g[b][n][p]: 64 × 64 tiles through LDS (coalesced both ways)
__global__ __launch_bounds__(256) void transpose_scale_kernel(const float* __restrict__ g, int N, int P, float scale,
                                                              float* __restrict__ gT) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const float* gb = g + (size_t)b * N * P;
  float* ob = gT + (size_t)b * N * P;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int n = n0 + ty + 4 * k, p = p0 + tx;
    tile[ty + 4 * k][tx] = (n < N && p < P) ? gb[(size_t)n * P + p] * scale : 0.0f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int p = p0 + ty + 4 * k, n = n0 + tx;
    if (n < N && p < P) ob[(size_t)p * N + n] = tile[tx][ty + 4 * k];
  }
}

// ------------------------------------------------------------------------------------ aggregate
struct LayerPtrs {
  const float* p[SKP_MAX_LAYERS];
};

// One block owns kAggP consecutive pixels × ALL N tokens.  In every (layer, b) slab those
// pixels are one contiguous run of kAggP·N floats, so the block streams it with 16-B loads in
// address order (no partially used cache lines at row seams), keeps the 32 slab sums in
// registers, and transposes the (pixel, token) tile through LDS for token-major stores.
constexpr int kAggP = 16;
constexpr int kAggThreads = 256;

template <int NV, int SPI, bool NT>  // float4 loads/thread/slab; slabs per iteration; non-temporal loads
__global__ __launch_bounds__(kAggThreads) void aggregate_kernel(LayerPtrs lp, int L, int BH, int RR, int N,
                                                                float count, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float tile[];   // kAggP*N floats
  const int p0 = blockIdx.x * kAggP;
  const int np = min(kAggP, RR - p0);
  const int flat = np * N;                     // valid floats in this block's run
  const int t = threadIdx.x;
  float4 acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int nslab = L * BH;
  for (int sl = 0; sl < nslab; sl += SPI) {
    float4 a[SPI][NV];
#pragma unroll
    for (int u = 0; u < SPI; ++u) {
      const int su = sl + u;
      const float* base = su < nslab ? lp.p[su / BH] + ((size_t)(su % BH) * RR + p0) * N : nullptr;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int f = 4 * (t + v * kAggThreads);
        if (base && f < flat) {
          if (NT) {
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v w = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(base + f));
            a[u][v] = make_float4(w.x, w.y, w.z, w.w);
          } else {
            a[u][v] = *reinterpret_cast<const float4*>(base + f);
          }
        } else {
          a[u][v] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < SPI; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        acc[v].x += a[u][v].x; acc[v].y += a[u][v].y; acc[v].z += a[u][v].z; acc[v].w += a[u][v].w;
      }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int f = 4 * (t + v * kAggThreads);
    if (f < flat) *reinterpret_cast<float4*>(tile + f) = acc[v];
  }
  __syncthreads();
  // tile[pl·N + n] -> out[n·RR + p0 + pl]: 16 lanes write one token's 64-B pixel run
  for (int e = t; e < np * N; e += kAggThreads) {
    const int n = e / np, pl = e - n * np;
    out[(size_t)n * RR + p0 + pl] = tile[pl * N + n] / count;
  }
}

// Fallback for unaligned layouts (N % 4 != 0 or misaligned base pointers): scalar loads.
__global__ __launch_bounds__(kAggThreads) void aggregate_scalar_kernel(LayerPtrs lp, int L, int BH, int RR, int N,
                                                                       float count, float* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * kAggThreads + threadIdx.x;   // (p, n) in slab order
  if (e >= (size_t)RR * N) return;
  const int p = e / N, n = e % N;
  float acc = 0.0f;
  for (int l = 0; l < L; ++l)
    for (int b = 0; b < BH; ++b) acc += lp.p[l][(size_t)b * RR * N + e];
  out[(size_t)n * RR + p] = acc / count;
}

__global__ __launch_bounds__(kThreads) void aggregate_index_kernel(LayerPtrs lp, int L, int BH, int RR, int N,
                                                                   const long long* __restrict__ idx, int n_out,
                                                                   float count, float* __restrict__ out) {
  const int p = blockIdx.x * kThreads + threadIdx.x;
  const int m = blockIdx.y;
  if (p >= RR) return;
  const long long tok = idx[m];
  float acc = 0.0f;
  for (int l = 0; l < L; ++l)
    for (int b = 0; b < BH; ++b) acc += lp.p[l][((size_t)b * RR + p) * N + tok];
  out[(size_t)m * RR + p] = acc / count;
}

// ------------------------------------------------------------------------------------ bilinear
__global__ void bilinear_kernel(const float* __restrict__ in, int C, int R, int Ro, float* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)C * Ro * Ro;
  if (e >= total) return;
  const int X = e % Ro, Y = (e / Ro) % Ro, c = e / ((size_t)Ro * Ro);
  const Taps2 ty = bilinear_taps(Y, R, Ro), tx = bilinear_taps(X, R, Ro);
  const float* p = in + (size_t)c * R * R;
  out[e] = ty.w0 * (tx.w0 * p[ty.i0 * R + tx.i0] + tx.w1 * p[ty.i0 * R + tx.i1]) +
           ty.w1 * (tx.w0 * p[ty.i1 * R + tx.i0] + tx.w1 * p[ty.i1 * R + tx.i1]);
}

// Adjoint, gather form (deterministic): input pixel (i, j) collects every output whose taps hit it.
__device__ __forceinline__ float bilinear_adj_weight(int dst, int src_i, int n_in, int n_out) {
  const Taps2 t = bilinear_taps(dst, n_in, n_out);
  float w = 0.0f;
  if (t.i0 == src_i) w += t.w0;
  if (t.i1 == src_i) w += t.w1;
  return w;
}

__global__ void bilinear_bwd_kernel(const float* __restrict__ gout, int C, int R, int Ro, float* __restrict__ gin) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)C * R * R;
  if (e >= total) return;
  const int j = e % R, i = (e / R) % R, c = e / ((size_t)R * R);
  const float ratio = (float)Ro / (float)R;
  const int lo_i = max(0, (int)floorf((i - 1.0f) * ratio) - 2), hi_i = min(Ro - 1, (int)ceilf((i + 2.0f) * ratio) + 2);
  const int lo_j = max(0, (int)floorf((j - 1.0f) * ratio) - 2), hi_j = min(Ro - 1, (int)ceilf((j + 2.0f) * ratio) + 2);
  const float* g = gout + (size_t)c * Ro * Ro;
  float acc = 0.0f;
  for (int Y = lo_i; Y <= hi_i; ++Y) {
    const float wy = bilinear_adj_weight(Y, i, R, Ro);
    if (wy == 0.0f) continue;
    float row = 0.0f;
    for (int X = lo_j; X <= hi_j; ++X) {
      const float wx = bilinear_adj_weight(X, j, R, Ro);
      if (wx != 0.0f) row += wx * g[(size_t)Y * Ro + X];
    }
    acc += wy * row;
  }
  gin[e] = acc;
}

template <int NQ>
void launch_fwd(const float* z, int BH, int s, int N, int R, float* attn, float2* stats, hipStream_t st) {
  const size_t lds = (size_t)s * NQ * 4 * WAVE * sizeof(float);
  const bool vec = (N % 4 == 0) && ((reinterpret_cast<uintptr_t>(z) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(attn) & 15) == 0);
  // Non-temporal stores measured faster at s = 32 (64 KiB LDS, 2 blocks/CU: 96 -> 75-84 us) and
  // slower at s = 16 (5 blocks/CU: 55 -> 80 us), N = 500, R = 128 (tools/kbench.py).
  const bool nts = lds > 48 * 1024;
  if (vec && nts)
    hipLaunchKernelGGL((capture_fwd_kernel<NQ, true, true>), dim3(BH * R), dim3(kThreads), lds, st, z, BH, s, N, R,
                       attn, stats);
  else if (vec)
    hipLaunchKernelGGL((capture_fwd_kernel<NQ, true>), dim3(BH * R), dim3(kThreads), lds, st, z, BH, s, N, R, attn, stats);
  else
    hipLaunchKernelGGL((capture_fwd_kernel<NQ, false>), dim3(BH * R), dim3(kThreads), lds, st, z, BH, s, N, R, attn, stats);
}

size_t bwd_rows_lds(int s, int N, int R, int CH);

template <int NT>
void launch_bwd_rows(const float* z, int BH, int s, int N, int R, int CH, const float* g, int group, long long sb,
                     long long sp, long long sn, float gscale, const float2* stats, float* ws, hipStream_t st) {
  const size_t lds = bwd_rows_lds(s, N, R, CH);
  const int share = sb == 0 ? BH : group;   // heads reading the same gradient rows
  hipLaunchKernelGGL((capture_bwd_rows_kernel<NT>), dim3(BH * R), dim3(kBwdThreads), lds, st, z, BH, s, N, R, CH, g,
                     group, sb, sp, sn, gscale, share, stats, ws);
}

int nt_for(int N);
size_t bwd_rows_lds(int s, int N, int R, int CH) {
  const size_t np = (size_t)nt_for(N) * kBwdThreads;
  return (s * np + (size_t)CH * (np + 4) + (size_t)R * 4 + (((size_t)R + 3) & ~(size_t)3)) * sizeof(float);
}

int nq_for(int N) {  // float4 quads per lane for the forward
  if (N <= 256) return 1;
  if (N <= 512) return 2;
  if (N <= 1024) return 4;
  return -1;
}

int nt_for(int N) {  // tokens per thread for the backward
  if (N <= 512) return 1;
  if (N <= 1024) return 2;
  return -1;
}

// chunk of output pixels for the backward: the largest multiple of 4 dividing R (enables the
// prefetched float4 gradient path) with which two blocks share a CU, else the largest that
// fits one CU's LDS.
int pick_chunk(int s, int N, int R) {
  for (size_t budget : {size_t(80) * 1024, size_t(160) * 1024}) {
    for (int ch = 16; ch >= 4; ch -= 4)
      if (R % ch == 0 && bwd_rows_lds(s, N, R, ch) <= budget) return ch;
    for (int ch = 16; ch >= 1; --ch)
      if (bwd_rows_lds(s, N, R, ch) <= budget) return ch;
  }
  return 1;
}

}  // namespace

extern "C" int skp_capture_fwd(const float* z_low, int BH, int s, int N, int R, float* attn, float* stats,
                               void* stream) {
  SKP_CHECK_ARG(z_low && attn, "null pointer");
  SKP_CHECK_ARG(BH > 0 && s > 0 && R > 0 && N > 0, "non-positive shape");
  const int nq = nq_for(N);
  SKP_CHECK_ARG(nq > 0, "N > 1024 tokens is not supported");
  SKP_CHECK_ARG((size_t)s * nq * 4 * WAVE * 4 <= 160 * 1024, "s*N too large for LDS");
  hipStream_t st = as_stream(stream);
  switch (nq) {
    case 1: launch_fwd<1>(z_low, BH, s, N, R, attn, reinterpret_cast<float2*>(stats), st); break;
    case 2: launch_fwd<2>(z_low, BH, s, N, R, attn, reinterpret_cast<float2*>(stats), st); break;
    default: launch_fwd<4>(z_low, BH, s, N, R, attn, reinterpret_cast<float2*>(stats), st); break;
  }
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_capture_bwd(const float* z_low, int BH, int s, int N, int R, const float* dattn, int group,
                               long long sb, long long sp, long long sn, float gscale, const float* stats,
                               float* dz_low, float* workspace, void* stream) {
  SKP_CHECK_ARG(z_low && dattn && dz_low && workspace, "null pointer");
  SKP_CHECK_ARG(group >= 1, "group must be >= 1");
  SKP_CHECK_ARG(BH > 0 && s > 0 && R > 0 && N > 0, "non-positive shape");
  SKP_CHECK_ARG(R <= 1024, "R > 1024 is not supported");
  SKP_CHECK_ARG(BH <= 65535, "BH > 65535");
  const int nt = nt_for(N);
  SKP_CHECK_ARG(nt > 0, "N > 1024 tokens is not supported");
  const int CH = pick_chunk(s, N, R);
  SKP_CHECK_ARG(bwd_rows_lds(s, N, R, CH) <= 160 * 1024, "s*N too large for LDS");
  hipStream_t st = as_stream(stream);
  const float2* st2 = reinterpret_cast<const float2*>(stats);
  if (nt == 1) launch_bwd_rows<1>(z_low, BH, s, N, R, CH, dattn, group, sb, sp, sn, gscale, st2, workspace, st);
  else launch_bwd_rows<2>(z_low, BH, s, N, R, CH, dattn, group, sb, sp, sn, gscale, st2, workspace, st);
  SKP_LAUNCH_CHECK();
  const int chunks = (int)(((long long)s * N + kColThreads - 1) / kColThreads);
  hipLaunchKernelGGL(capture_bwd_cols_kernel, dim3(chunks, BH), dim3(kColThreads), 0, st, workspace, BH, s, N, R,
                     dz_low);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

namespace {
int maps_qpl(int N) {   // float4 quads per lane (16 lanes per pixel): Np = 64·QPL >= N
  if (N <= 64) return 1;
  if (N <= 128) return 2;
  if (N <= 256) return 4;
  if (N <= 512) return 8;
  if (N <= 1024) return 16;
  return -1;
}

// floats per V buffer: the widest layer's nc × Np, and at least half the store tile (P × 132)
int maps_vstride(const int* sizes, int L, int R, int qpl, int waves) {
  const int P = waves * maps_pxw(qpl);
  const int Np = 64 * qpl;
  int ncmax = 1;
  for (int l = 0; l < L; ++l) {   // columns one P-pixel chunk can touch: ⌈P·s/R⌉ + 4, at most s
    const int s = sizes[l];
    ncmax = std::max(ncmax, std::min(s, (int)(((long long)P * s + R - 1) / R) + 4));
  }
  const int v = ncmax * Np, tile = P * (128 + 4);
  return (std::max(v, (tile + 1) / 2) + 3) & ~3;
}

size_t maps_lds(int vstride, int qpl, int waves) {   // [2][P] taps ×2 + [2][vstride] V
  return (16 * (size_t)waves * maps_pxw(qpl) + 2 * (size_t)vstride) * sizeof(float);
}

// 8-wave workgroups, a persistent grid of two per CU walking their XCD's rows in step (1003 vs
// 1013 µs and FETCH_SIZE 955 vs 1070 MB against one job per workgroup,
// profiles/r03ad_maps_persist_ab.txt; 4- and 16-wave workgroups measured slower,
// profiles/r05w_maps_waves_ab.txt)
constexpr int kMapWaves = 8;

template <int QPL>
void launch_maps(const CapLayers& cl, int L, int B, int H, int N, int R, int vstride, size_t lds, float* maps,
                 hipStream_t st) {
  constexpr int WAVES = kMapWaves;
  const int P = WAVES * maps_pxw(QPL);
  const int nchunks = (R + P - 1) / P;
  const int total = B * R * nchunks;
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return std::max(8, n / 8 * 8);
  }();
  const int grid = std::min(8 * ((total + 7) / 8), (16 / WAVES) * ncu);   // multiple of 8
  hipLaunchKernelGGL((capture_maps_kernel<QPL, WAVES>), dim3(grid), dim3(WAVES * WAVE), lds, st, cl, L, B, H, N, R,
                     nchunks, vstride, (float)L * (float)H, maps);
}
}  // namespace

extern "C" int skp_capture_maps_fwd(const float* const* z_low, const int* sizes, int L, int B, int H, int N, int R,
                                    float* maps, float* const* stats, void* stream) {
  SKP_CHECK_ARG(z_low && sizes && maps, "null pointer");
  SKP_CHECK_ARG(L > 0 && L <= SKP_MAX_LAYERS, "L out of range");
  SKP_CHECK_ARG(B > 0 && H > 0 && N > 0 && R > 0, "non-positive shape");
  SKP_CHECK_ARG((long long)B * R * R <= (1LL << 31) && (long long)B * H <= 65535, "shape too large");
  const int qpl = maps_qpl(N);
  SKP_CHECK_ARG(qpl > 0, "N > 1024 tokens is not supported");
  CapLayers cl{};
  bool aligned = (N % 4) == 0;
  for (int l = 0; l < L; ++l) {
    SKP_CHECK_ARG(z_low[l], "null layer pointer");
    SKP_CHECK_ARG(sizes[l] > 0 && sizes[l] <= R, "layer size must be in [1, R]");
    cl.z[l] = z_low[l];
    cl.s[l] = sizes[l];
    cl.sc[l] = (float)sizes[l] / (float)R;
    cl.stats[l] = stats ? reinterpret_cast<float2*>(stats[l]) : nullptr;
    aligned = aligned && ((reinterpret_cast<uintptr_t>(z_low[l]) & 15) == 0);
  }
  SKP_CHECK_ARG(aligned || (N % 4) != 0, "z_low pointers must be 16-B aligned");
  hipStream_t st = as_stream(stream);
  const int vstride = maps_vstride(sizes, L, R, qpl, kMapWaves);
  const size_t lds = maps_lds(vstride, qpl, kMapWaves);
  SKP_CHECK_ARG(lds <= 160 * 1024, "s*N too large for LDS");
  switch (qpl) {
    case 1: launch_maps<1>(cl, L, B, H, N, R, vstride, lds, maps, st); break;
    case 2: launch_maps<2>(cl, L, B, H, N, R, vstride, lds, maps, st); break;
    case 4: launch_maps<4>(cl, L, B, H, N, R, vstride, lds, maps, st); break;
    case 8: launch_maps<8>(cl, L, B, H, N, R, vstride, lds, maps, st); break;
    default: launch_maps<16>(cl, L, B, H, N, R, vstride, lds, maps, st); break;
  }
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

namespace {
template <int NQ>
void launch_bwd_row(const float* z, int B, int H, int s, int N, int R, const float* gT, const float* stats, float* ws,
                    hipStream_t st) {
  const long long total = (long long)B * H * R;
  const long long blocks = (total + kRowThreads / WAVE - 1) / (kRowThreads / WAVE);
  const long long grid = 8 * ((blocks + 7) / 8);
  const float2* st2 = reinterpret_cast<const float2*>(stats);
  const size_t lds = bwd_row_lds(R, NQ);
  if (stats)
    hipLaunchKernelGGL((capture_bwd_row_kernel<NQ, true>), dim3((unsigned)grid), dim3(kRowThreads), lds, st, z, B, H, s,
                       N, R, gT, st2, ws);
  else
    hipLaunchKernelGGL((capture_bwd_row_kernel<NQ, false>), dim3((unsigned)grid), dim3(kRowThreads), lds, st, z, B, H, s,
                       N, R, gT, st2, ws);
}
}  // namespace

extern "C" int skp_capture_maps_bwd(const float* const* z_low, const int* sizes, int L, int B, int H, int N, int R,
                                    const float* dmaps, float gscale, const float* const* stats, float* const* dz_low,
                                    float* workspace, void* stream) {
  SKP_CHECK_ARG(z_low && sizes && dmaps && dz_low && workspace, "null pointer");
  SKP_CHECK_ARG(L > 0 && L <= SKP_MAX_LAYERS, "L out of range");
  SKP_CHECK_ARG(B > 0 && H > 0 && N > 0 && R > 0, "non-positive shape");
  SKP_CHECK_ARG(N % 4 == 0, "N must be a multiple of 4 (use skp_capture_bwd)");
  SKP_CHECK_ARG(N <= 1024, "N > 1024 tokens is not supported");
  SKP_CHECK_ARG(R <= 1024, "R > 1024 is not supported (capture_bwd_cols_kernel tap tables)");
  SKP_CHECK_ARG(bwd_row_lds(R, N <= 256 ? 1 : (N <= 512 ? 2 : 4)) <= 160 * 1024, "R * N too large for LDS");
  SKP_CHECK_ARG((long long)B * H <= 65535 && (long long)B * H * R < (1LL << 31), "shape too large");
  SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "workspace must be 16-B aligned");
  int smax = 0;
  for (int l = 0; l < L; ++l) {
    SKP_CHECK_ARG(z_low[l] && dz_low[l], "null layer pointer");
    SKP_CHECK_ARG(sizes[l] > 0 && sizes[l] <= R && sizes[l] <= 1024, "layer size must be in [1, R]");
    SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(z_low[l]) & 15) == 0, "z_low pointers must be 16-B aligned");
    smax = std::max(smax, sizes[l]);
  }
  hipStream_t st = as_stream(stream);
  const int P = R * R;
  float* gT = workspace;                                   // (B, R², N)
  float* ws = workspace + (size_t)B * P * N;               // (B·H, R, s, N) row partials, reused per layer
  if ((P % 4) == 0 && (reinterpret_cast<uintptr_t>(dmaps) & 15) == 0)   // N % 4 == 0 is checked above
    hipLaunchKernelGGL(transpose_scale4_kernel, dim3((P + 63) / 64, (N + 63) / 64, B), dim3(256), 0, st, dmaps, N, P,
                       gscale, gT);
  else
    hipLaunchKernelGGL(transpose_scale_kernel, dim3((P + 63) / 64, (N + 63) / 64, B), dim3(256), 0, st, dmaps, N, P,
                       gscale, gT);
  SKP_LAUNCH_CHECK();
  const int nq = N / 4;
  for (int l = 0; l < L; ++l) {
    const int s = sizes[l];
    // the row kernel reads the stats as float4 pixel pairs: 16-B aligned rows need an even R
    const float* stl = (stats && (R % 2) == 0) ? stats[l] : nullptr;
    if (nq <= 64) launch_bwd_row<1>(z_low[l], B, H, s, N, R, gT, stl, ws, st);
    else if (nq <= 128) launch_bwd_row<2>(z_low[l], B, H, s, N, R, gT, stl, ws, st);
    else launch_bwd_row<4>(z_low[l], B, H, s, N, R, gT, stl, ws, st);
    SKP_LAUNCH_CHECK();
    // (a float4 form of this kernel measured the same 81 µs: it streams the row partials at
    // ≈4.7 TB/s either way)
    const int chunks = (int)(((long long)s * N + kColThreads - 1) / kColThreads);
    hipLaunchKernelGGL(capture_bwd_cols_kernel, dim3(chunks, B * H), dim3(kColThreads), 0, st, ws, B * H, s, N, R,
                       dz_low[l]);
    SKP_LAUNCH_CHECK();
  }
  (void)smax;
  return SKP_OK;
}

extern "C" int skp_aggregate(const float* const* layers, int L, int BH, int RR, int N, const long long* indices,
                             int n_out, float* out, void* stream) {
  SKP_CHECK_ARG(layers && out, "null pointer");
  SKP_CHECK_ARG(L > 0 && L <= SKP_MAX_LAYERS, "L out of range");
  SKP_CHECK_ARG(BH > 0 && RR > 0 && N > 0, "non-positive shape");
  LayerPtrs lp{};
  bool aligned = (N % 4) == 0;
  for (int l = 0; l < L; ++l) {
    SKP_CHECK_ARG(layers[l], "null layer pointer");
    lp.p[l] = layers[l];
    aligned = aligned && ((reinterpret_cast<uintptr_t>(layers[l]) & 15) == 0);
  }
  const float count = (float)L * (float)BH;
  hipStream_t st = as_stream(stream);
  if (indices) {
    SKP_CHECK_ARG(n_out > 0, "n_out must be positive with indices");
    hipLaunchKernelGGL(aggregate_index_kernel, dim3((RR + kThreads - 1) / kThreads, n_out), dim3(kThreads), 0, st, lp,
                       L, BH, RR, N, indices, n_out, count, out);
  } else {
    const int nv = (kAggP * N + 4 * kAggThreads - 1) / (4 * kAggThreads);
    const bool vec = aligned && (RR % kAggP == 0) && nv <= 8;
    const size_t lds = (size_t)kAggP * N * sizeof(float);
    const dim3 grid((RR + kAggP - 1) / kAggP);
    if (!vec) {
      hipLaunchKernelGGL(aggregate_scalar_kernel, dim3(((size_t)RR * N + kAggThreads - 1) / kAggThreads),
                         dim3(kAggThreads), 0, st, lp, L, BH, RR, N, count, out);
    } else {
      // 2 slabs per iteration, non-temporal 16-B loads (read-once stream: +11% over cached loads,
      // 6.0 vs 5.35 TB/s on N=500 / R=128 / 4 layers × 8 heads, tools/kbench.py)
#define SKP_AGG(NV) \
  hipLaunchKernelGGL((aggregate_kernel<NV, 2, true>), grid, dim3(kAggThreads), lds, st, lp, L, BH, RR, N, count, out)
      if (nv <= 1) SKP_AGG(1);
      else if (nv <= 2) SKP_AGG(2);
      else if (nv <= 4) SKP_AGG(4);
      else SKP_AGG(8);
#undef SKP_AGG
    }
  }
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_resize_bilinear(const float* in, int C, int R, int Ro, float* out, void* stream) {
  SKP_CHECK_ARG(in && out, "null pointer");
  SKP_CHECK_ARG(C > 0 && R > 0 && Ro > 0, "non-positive shape");
  const size_t total = (size_t)C * Ro * Ro;
  hipLaunchKernelGGL(bilinear_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), in, C, R, Ro, out);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_resize_bilinear_bwd(const float* gout, int C, int R, int Ro, float* gin, void* stream) {
  SKP_CHECK_ARG(gout && gin, "null pointer");
  SKP_CHECK_ARG(C > 0 && R > 0 && Ro > 0, "non-positive shape");
  const size_t total = (size_t)C * R * R;
  hipLaunchKernelGGL(bilinear_bwd_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), gout, C, R, Ro,
                     gin);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
