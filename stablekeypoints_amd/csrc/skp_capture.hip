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
// horizontal adjoint into per-wave register accumulators (deterministic, no atomics),
// writes row partials, and a second kernel applies the vertical adjoint.
#include "skp_common.h"

using namespace skp;

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / WAVE;

// ------------------------------------------------------------------------------------ fwd
template <int NCH>
__global__ __launch_bounds__(kThreads) void capture_fwd_kernel(const float* __restrict__ z, int BH, int s, int N,
                                                               int R, float* __restrict__ attn) {
  extern __shared__ __attribute__((aligned(16))) float V[];
  constexpr int Np = NCH * WAVE;
  // block -> (b, y) with b fastest: consecutive blocks (one per XCD under round-robin
  // dispatch) take different heads, so each XCD's L2 keeps the z_low of the heads it serves.
  const int b = blockIdx.x % BH;
  const int y = blockIdx.x / BH;
  const Taps4 ty = bicubic_taps(y, s, R);
  const float* zb = z + (size_t)b * s * s * N;
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
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* orow = attn + ((size_t)b * R * R + (size_t)y * R) * N;
  for (int x = wid; x < R; x += kWaves) {
    const Taps4 tx = bicubic_taps(x, s, R);
    float zc[NCH];
    float m = -INFINITY;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int n = c * WAVE + lane;
      float v = tx.w[0] * V[tx.i[0] * Np + n];
      v += tx.w[1] * V[tx.i[1] * Np + n];
      v += tx.w[2] * V[tx.i[2] * Np + n];
      v += tx.w[3] * V[tx.i[3] * Np + n];
      zc[c] = n < N ? v : -INFINITY;
      m = fmaxf(m, zc[c]);
    }
    m = wave_max(m);
    float ssum = 0.0f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int n = c * WAVE + lane;
      const float e = n < N ? expf(zc[c] - m) : 0.0f;
      zc[c] = e;
      ssum += e;
    }
    ssum = wave_sum(ssum);
    float* o = orow + (size_t)x * N;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int n = c * WAVE + lane;
      if (n < N) o[n] = zc[c] / ssum;
    }
  }
}

// ------------------------------------------------------------------------------------ bwd
// Phase A: one block per (b, y).  Wave w owns low-res columns j in [w·JPW, (w+1)·JPW).
constexpr int kChunk = 16;  // output pixels per staged chunk

template <int NCH, int JPW>
__global__ __launch_bounds__(kThreads) void capture_bwd_rows_kernel(const float* __restrict__ z, int BH, int s,
                                                                    int N, int R, const float* __restrict__ g,
                                                                    long long sb, long long sp, long long sn,
                                                                    float gscale, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int Np = NCH * WAVE;
  float* V = lds;               // s × Np
  float* G = lds + s * Np;      // kChunk × Np
  const int b = blockIdx.x % BH;
  const int y = blockIdx.x / BH;
  const Taps4 ty = bicubic_taps(y, s, R);
  const float* zb = z + (size_t)b * s * s * N;
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
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int jbase = wid * JPW;
  float acc[JPW][NCH];
#pragma unroll
  for (int jj = 0; jj < JPW; ++jj)
#pragma unroll
    for (int c = 0; c < NCH; ++c) acc[jj][c] = 0.0f;

  const float* gb = g + (long long)b * sb + (long long)y * R * sp;
  for (int x0 = 0; x0 < R; x0 += kChunk) {
    __syncthreads();  // previous chunk's G fully consumed (and V ready on the first pass)
    if (sn == 1) {
      for (int e = threadIdx.x; e < kChunk * Np; e += kThreads) {
        const int xx = e / Np, n = e - xx * Np;
        const int x = x0 + xx;
        G[e] = (n < N && x < R) ? gb[(long long)x * sp + n] * gscale : 0.0f;
      }
    } else {
      for (int e = threadIdx.x; e < kChunk * Np; e += kThreads) {
        const int n = e / kChunk, xx = e - n * kChunk;
        const int x = x0 + xx;
        G[xx * Np + n] = (n < N && x < R) ? gb[(long long)x * sp + (long long)n * sn] * gscale : 0.0f;
      }
    }
    __syncthreads();
    for (int xx = wid; xx < kChunk; xx += kWaves) {
      const int x = x0 + xx;
      if (x >= R) break;
      const Taps4 tx = bicubic_taps(x, s, R);
      float a[NCH];
      float m = -INFINITY;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int n = c * WAVE + lane;
        float v = tx.w[0] * V[tx.i[0] * Np + n];
        v += tx.w[1] * V[tx.i[1] * Np + n];
        v += tx.w[2] * V[tx.i[2] * Np + n];
        v += tx.w[3] * V[tx.i[3] * Np + n];
        a[c] = n < N ? v : -INFINITY;
        m = fmaxf(m, a[c]);
      }
      m = wave_max(m);
      float ssum = 0.0f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int n = c * WAVE + lane;
        a[c] = n < N ? expf(a[c] - m) : 0.0f;
        ssum += a[c];
      }
      ssum = wave_sum(ssum);
      float dot = 0.0f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        a[c] = a[c] / ssum;
        dot += a[c] * G[xx * Np + c * WAVE + lane];
      }
      dot = wave_sum(dot);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int n = c * WAVE + lane;
        G[xx * Np + n] = a[c] * (G[xx * Np + n] - dot);
      }
    }
    __syncthreads();
    // horizontal adjoint of this chunk into the wave's own columns (fixed order -> deterministic)
    for (int xx = 0; xx < kChunk; ++xx) {
      const int x = x0 + xx;
      if (x >= R) break;
      const Taps4 tx = bicubic_taps(x, s, R);
#pragma unroll
      for (int jj = 0; jj < JPW; ++jj) {
        const int j = jbase + jj;
        float w = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) w += (tx.i[k] == j) ? tx.w[k] : 0.0f;
        if (w != 0.0f && j < s) {
#pragma unroll
          for (int c = 0; c < NCH; ++c) acc[jj][c] += w * G[xx * Np + c * WAVE + lane];
        }
      }
    }
  }
  // ws layout (BH, R, s, N): row partials of the vertical adjoint's input
  float* wrow = ws + ((size_t)b * R + y) * (size_t)s * N;
#pragma unroll
  for (int jj = 0; jj < JPW; ++jj) {
    const int j = jbase + jj;
    if (j >= s) continue;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int n = c * WAVE + lane;
      if (n < N) wrow[(size_t)j * N + n] = acc[jj][c];
    }
  }
}

// Phase B: dz[b][i·s + j][n] = Σ_y wy(y→i) · ws[b][y][j][n]; one block per (b, i).
__global__ __launch_bounds__(kThreads) void capture_bwd_cols_kernel(const float* __restrict__ ws, int BH, int s,
                                                                    int N, int R, float* __restrict__ dz) {
  __shared__ int ylist[1024];
  __shared__ float wlist[1024];
  __shared__ int ny;
  const int b = blockIdx.x % BH;
  const int i = blockIdx.x / BH;
  if (threadIdx.x == 0) {
    int cnt = 0;
    for (int y = 0; y < R; ++y) {
      const Taps4 ty = bicubic_taps(y, s, R);
      float w = 0.0f;
      bool hit = false;
      for (int k = 0; k < 4; ++k)
        if (ty.i[k] == i) { w += ty.w[k]; hit = true; }
      if (hit && w != 0.0f) { ylist[cnt] = y; wlist[cnt] = w; ++cnt; }
    }
    ny = cnt;
  }
  __syncthreads();
  const int cnt = ny;
  const size_t plane = (size_t)s * N;
  const float* wb = ws + (size_t)b * R * plane;
  float* out = dz + ((size_t)b * s * s + (size_t)i * s) * N;
  for (int e = threadIdx.x; e < s * N; e += kThreads) {
    float acc = 0.0f;
    for (int t = 0; t < cnt; ++t) acc += wlist[t] * wb[(size_t)ylist[t] * plane + e];
    out[e] = acc;
  }
}

// ------------------------------------------------------------------------------------ aggregate
struct LayerPtrs {
  const float* p[SKP_MAX_LAYERS];
};

constexpr int kTileP = 64, kTileN = 64;

template <bool VEC>
__global__ __launch_bounds__(kThreads) void aggregate_kernel(LayerPtrs lp, int L, int BH, int RR, int N,
                                                             float count, float* __restrict__ out) {
  __shared__ float T[kTileN][kTileP + 1];
  const int p0 = blockIdx.x * kTileP, n0 = blockIdx.y * kTileN;
  const int t = threadIdx.x, q = t & 15, r = t >> 4;
  const int n = n0 + 4 * q;
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = 0.0f;
  for (int l = 0; l < L; ++l) {
    const float* base = lp.p[l];
#pragma unroll 2
    for (int b = 0; b < BH; ++b) {
      const float* bb = base + (size_t)b * RR * N;
      float4 v[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int p = p0 + r + 16 * a;
        v[a] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (p < RR) {
          const float* src = bb + (size_t)p * N + n;
          if (VEC) {
            if (n + 3 < N) v[a] = *reinterpret_cast<const float4*>(src);
            else {
              if (n < N) v[a].x = src[0];
              if (n + 1 < N) v[a].y = src[1];
              if (n + 2 < N) v[a].z = src[2];
            }
          } else {
            if (n < N) v[a].x = src[0];
            if (n + 1 < N) v[a].y = src[1];
            if (n + 2 < N) v[a].z = src[2];
            if (n + 3 < N) v[a].w = src[3];
          }
        }
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        acc[a][0] += v[a].x;
        acc[a][1] += v[a].y;
        acc[a][2] += v[a].z;
        acc[a][3] += v[a].w;
      }
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) T[4 * q + c][r + 16 * a] = acc[a][c];
  __syncthreads();
  const int pl = t & 63;
  for (int nl = t >> 6; nl < kTileN; nl += kThreads / 64) {
    const int nn = n0 + nl, pp = p0 + pl;
    if (nn < N && pp < RR) out[(size_t)nn * RR + pp] = T[nl][pl] / count;
  }
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

template <int NCH>
int launch_fwd(const float* z, int BH, int s, int N, int R, float* attn, hipStream_t st) {
  const size_t lds = (size_t)s * NCH * WAVE * sizeof(float);
  hipLaunchKernelGGL(capture_fwd_kernel<NCH>, dim3(BH * R), dim3(kThreads), lds, st, z, BH, s, N, R, attn);
  return 0;
}

template <int NCH, int JPW>
void launch_bwd_rows(const float* z, int BH, int s, int N, int R, const float* g, long long sb, long long sp,
                     long long sn, float gscale, float* ws, hipStream_t st) {
  const size_t lds = (size_t)(s + kChunk) * NCH * WAVE * sizeof(float);
  hipLaunchKernelGGL((capture_bwd_rows_kernel<NCH, JPW>), dim3(BH * R), dim3(kThreads), lds, st, z, BH, s, N, R, g,
                     sb, sp, sn, gscale, ws);
}

int nch_for(int N) {
  if (N <= 64) return 1;
  if (N <= 128) return 2;
  if (N <= 256) return 4;
  if (N <= 512) return 8;
  if (N <= 1024) return 16;
  return -1;
}

}  // namespace

extern "C" int skp_capture_fwd(const float* z_low, int BH, int s, int N, int R, float* attn, void* stream) {
  SKP_CHECK_ARG(z_low && attn, "null pointer");
  SKP_CHECK_ARG(BH > 0 && s > 0 && R > 0 && N > 0, "non-positive shape");
  const int nch = nch_for(N);
  SKP_CHECK_ARG(nch > 0, "N > 1024 tokens is not supported");
  SKP_CHECK_ARG((size_t)s * nch * WAVE * 4 <= 160 * 1024, "s*N too large for LDS");
  hipStream_t st = as_stream(stream);
  switch (nch) {
    case 1: launch_fwd<1>(z_low, BH, s, N, R, attn, st); break;
    case 2: launch_fwd<2>(z_low, BH, s, N, R, attn, st); break;
    case 4: launch_fwd<4>(z_low, BH, s, N, R, attn, st); break;
    case 8: launch_fwd<8>(z_low, BH, s, N, R, attn, st); break;
    default: launch_fwd<16>(z_low, BH, s, N, R, attn, st); break;
  }
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_capture_bwd(const float* z_low, int BH, int s, int N, int R, const float* dattn, long long sb,
                               long long sp, long long sn, float gscale, float* dz_low, float* workspace,
                               void* stream) {
  SKP_CHECK_ARG(z_low && dattn && dz_low && workspace, "null pointer");
  SKP_CHECK_ARG(BH > 0 && s > 0 && R > 0 && N > 0, "non-positive shape");
  SKP_CHECK_ARG(R <= 1024, "R > 1024 is not supported");
  const int nch = nch_for(N);
  SKP_CHECK_ARG(nch > 0, "N > 1024 tokens is not supported");
  SKP_CHECK_ARG(s <= 64, "s > 64 is not supported");
  SKP_CHECK_ARG((size_t)(s + kChunk) * nch * WAVE * 4 <= 160 * 1024, "s*N too large for LDS");
  hipStream_t st = as_stream(stream);
  const int jpw = (s + kWaves - 1) / kWaves;  // low-res columns per wave
#define SKP_BWD_J(NC)                                                                            \
  if (jpw <= 1) launch_bwd_rows<NC, 1>(z_low, BH, s, N, R, dattn, sb, sp, sn, gscale, workspace, st); \
  else if (jpw <= 2) launch_bwd_rows<NC, 2>(z_low, BH, s, N, R, dattn, sb, sp, sn, gscale, workspace, st); \
  else if (jpw <= 4) launch_bwd_rows<NC, 4>(z_low, BH, s, N, R, dattn, sb, sp, sn, gscale, workspace, st); \
  else if (jpw <= 8) launch_bwd_rows<NC, 8>(z_low, BH, s, N, R, dattn, sb, sp, sn, gscale, workspace, st); \
  else launch_bwd_rows<NC, 16>(z_low, BH, s, N, R, dattn, sb, sp, sn, gscale, workspace, st);
  switch (nch) {
    case 1: SKP_BWD_J(1) break;
    case 2: SKP_BWD_J(2) break;
    case 4: SKP_BWD_J(4) break;
    case 8: SKP_BWD_J(8) break;
    default: SKP_BWD_J(16) break;
  }
#undef SKP_BWD_J
  SKP_LAUNCH_CHECK();
  hipLaunchKernelGGL(capture_bwd_cols_kernel, dim3(BH * s), dim3(kThreads), 0, st, workspace, BH, s, N, R, dz_low);
  SKP_LAUNCH_CHECK();
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
    dim3 grid((RR + kTileP - 1) / kTileP, (N + kTileN - 1) / kTileN);
    if (aligned)
      hipLaunchKernelGGL(aggregate_kernel<true>, grid, dim3(kThreads), 0, st, lp, L, BH, RR, N, count, out);
    else
      hipLaunchKernelGGL(aggregate_kernel<false>, grid, dim3(kThreads), 0, st, lp, L, BH, RR, N, count, out);
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
