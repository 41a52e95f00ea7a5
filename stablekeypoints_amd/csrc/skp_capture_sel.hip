// Backward of the fused capture + per-image aggregate (skp_capture_maps_fwd) for a SPARSE map
// gradient: the token-optimisation loss only reads maps[b, tok] for the few tokens the
// selection kept (reference optimize.py:403-424: sharpening and equivariance losses on
// top_embedding_indices), so the map gradient of image b is nonzero only in K token rows.
//
// Per layer l, head bh = b·H + h, output pixel p and token n, with a = softmax_n(z(p)) rebuilt
// from the forward's per-pixel (max, 1/Σ) and g the (scaled) map gradient:
//     dZ[p, n] = a[p, n]·(g[p, n] − dot[p]),   dot[p] = Σ_n a[p, n]·g[p, n] = Σ_k a[p, tok_k]·g_k[p]
// which splits into
//   - a sparse part  a[p, tok_k]·g_k[p]   (K tokens; e_k[p] below), and
//   - a dense part  −dot[p]·a[p, n]       (every token, but with ONE scalar per pixel instead of a
//                                           gradient row: no (B, N, R²) gradient, no transpose, no
//                                           per-pixel 500-token reduction).
// dz_low = bicubicᵀ(dZ) (the adjoint of the s→R upsampling, ptp_utils.py:513-529).
//
// Kernels (per layer):
//   sel_gather   zsel[bh][q][k] = z_low[bh][q][tok_k]                         (the selected logits)
//   sel_doth     per (bh, row y): a_k, e_k = a_k·g_k and dot → pix[bh][p] = (mb, −dot) with
//                mb = log2(1/Σ) − max·log2e, so a = exp2(z·log2e + mb); the row's e_k stay in LDS and
//                leave as the horizontal half of bicubicᵀ, Hs[bh][k][y][j] (R·s floats, not R²)
//   sel_adjv     per (bh, k): es[bh][k] = the vertical half of bicubicᵀ over Hs (R × s → s²),
//                deterministic
//   sel_dense    per (bh, 128-token chunk): the dense part's adjoint, plus es at the selected tokens
// sel_dense is the hot kernel.  One workgroup = R/PW bands of 64 (or, at R/s = 4, 32) lanes; band
// w owns output columns [PW·w, PW·w + PW) of every row and lanes own token pairs (packed f32:
// v_pk_fma).  With R = S·RATIO
// (RATIO a power of two, 4..16) the bicubic taps of a wave's pixels relative to its band are the
// same for every wave and every row group, so the horizontal taps, the pixel loop and the register
// indices are compile-time; the tap weights (RATIO distinct sets) sit in SGPRs, and so do the
// per-pixel (mb, d) pairs.  Registers per lane hold
//   Zw[4][NC]  the 4 low-res z rows the current output rows interpolate (band columns),
//   V[NC]      their vertical pass for the current row,   Hs[NC] its horizontal adjoint,
//   acc[4][NC] the vertical adjoint of the 4 low-res rows the current rows touch.
// A low-res row is complete when the rows' first tap moves past it: the waves' band partials are
// merged through LDS in a fixed order (bands overlap by NC − 16/RATIO columns; virtual columns
// and rows past the edges fold into 0 / s−1 exactly as torch's clamped taps), the sparse es is
// added at the selected tokens, and the row leaves as coalesced 512-B token runs.
// Every output element has one owner and a fixed summation order: deterministic, no atomics.
#include <algorithm>
#include <vector>

#include "skp_common.h"

using namespace skp;

namespace {

constexpr float L2E = 1.4426950408889634f;
constexpr int SEL_MAXK = 32;

typedef float f2 __attribute__((ext_vector_type(2)));

// first bicubic tap (before clamping) of output index t relative to its ratio group:
// floor((t + 0.5)/RATIO − 0.5) − 1, exact in integers for a power-of-two RATIO
constexpr int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
constexpr int lo_rel(int t, int ratio) { return floor_div(2 * t + 1 - ratio, 2 * ratio) - 1; }

// ------------------------------------------------------------------------------ sel_gather
// The small per-layer kernels (sel_gather, sel_dot, sel_adj) each run every layer in ONE launch:
// per-layer pointers and sizes by value, the layer found from the block / element index (12 short
// launches per step → 3, so no launch tail per layer).
struct SelSmall {
  const float* z[SKP_MAX_LAYERS];
  const float2* stats[SKP_MAX_LAYERS];
  int s[SKP_MAX_LAYERS];
  long long zoff[SKP_MAX_LAYERS + 1];   // zsel prefix offsets (floats): Σ BH·s²·K
};

__global__ void sel_gather_kernel(SelSmall t, int L, int BH, int N, int H, const long long* __restrict__ tok, int K,
                                  float* __restrict__ zsel) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= t.zoff[L]) return;
  int l = 0;
  while (l + 1 < L && e >= t.zoff[l + 1]) ++l;
  const long long le = e - t.zoff[l];
  const int SS = t.s[l] * t.s[l];
  const int k = (int)(le % K);
  const long long bq = le / K;   // bh·SS + q
  const int bh = (int)(bq / SS);
  const long long tk = tok[(long long)(bh / H) * K + k];
  zsel[e] = (tk >= 0 && tk < N) ? t.z[l][bq * N + tk] : 0.0f;
}

// The per-pixel pair sel_dense reads: (mb, d) with d = −dot and a = exp2(z·log2e + mb).  With
// SKP_SEL_DFOLD (default) |d| is folded into the exponent, (mb + log2|d|, d): sel_dense then gets
// a·|d| from its exp2 and d's sign from its tap weights' sign bits (scalar xors), one packed
// multiply per (pixel, token pair) less (d = 0 gives exp2(−inf) = 0).
#ifndef SKP_SEL_DFOLD
#define SKP_SEL_DFOLD 1
#endif
__device__ __forceinline__ float2 sel_pix(float mb, float dot) {
#if SKP_SEL_DFOLD
  return make_float2(mb + __builtin_amdgcn_logf(fabsf(dot)), -dot);   // v_log_f32 = log2
#else
  return make_float2(mb, -dot);
#endif
}

// output indices whose taps can reach low-res index j: src ∈ [j − 2, j + 2) (clamped edges included)
__device__ __forceinline__ void adj_range(int j, int S, int R, int& lo, int& hi) {
  const float r = (float)R / (float)S;
  lo = max(0, (int)floorf((j - 1.5f) * r - 0.5f) - 1);
  hi = min(R - 1, (int)ceilf((j + 2.5f) * r - 0.5f) + 1);
  if (j == 0) lo = 0;
  if (j == S - 1) hi = R - 1;
}

// ------------------------------------------------------------------------------ sel_doth
// sel_dot with the horizontal half of the sparse part's bicubicᵀ fused in (r05): the row's e_k stay
// in LDS and leave as Hs[l][bh][k][y][j] = Σ_x A[j][x]·e_k[y][x] (R·s floats per (bh, k) instead
// of E's R², so E's write + re-read — 2 × 168 MB at the bench shape — is gone; sel_adjv does the
// vertical half).  One block per (layer, bh, y), R threads (R ≤ 256).  The kernel is a chain of
// short phases (staging → pixels → columns) over 32 K blocks at the bench shape, so its time is
// set by how many blocks a CU holds and by each block's exposed load latency: r06 issues every
// global load of the block (the staging's selected logits, the pixel's stats and its K gradient
// values) before the first barrier, keeps the LDS at ≈ 9 KB (pads of 3.5·RATIO, no column buffer)
// and writes the Hs values straight from the column phase (2 barriers instead of 3).
// At R = RATIO·s (RATIO a power of two) virtual column c takes its taps from the 4·RATIO pixels
// x = RATIO·(c − 2) + RATIO/2 + t, t ∈ [0, 4·RATIO), with weight W[t] = w_{3 − t/RATIO} of pixel
// phase (RATIO/2 + t) mod RATIO: one fixed filter for every column, so column c is a 4·RATIO-tap dot
// product against the row's e (zero-padded past both edges), and the clamped edge columns add their
// virtual columns −2, −1, 0 / S − 1, S, S + 1 in that order.  Per column the terms run x ascending
// from 0 — the summation order of a rolling window over the row (r04's sel_adjw, which took E
// through HBM; r05 measured Hs and es bit-identical to it before it was removed in r06).
template <int RMAX>
constexpr int doth_pad() { return 4 * RMAX; }   // zero floats each side of a row's e (≥ 3.5·RATIO)

// virtual column c = cv − 2 of e row k: Σ_t W[t]·e_k[RATIO·(c − 2) + RATIO/2 + t]
template <int RATIO, int PAD>
__device__ __forceinline__ float doth_column(const float* __restrict__ W, const float* __restrict__ Ek, int cv) {
  constexpr int NT = 4 * RATIO;
  const float* src = Ek + PAD + RATIO / 2 - 4 * RATIO + RATIO * cv;
  float a = 0.0f;
  if constexpr (RATIO >= 8) {   // 16-B aligned runs (EP, PAD and RATIO/2 multiples of 4)
    const float4* s4 = reinterpret_cast<const float4*>(src);
    const float4* w4 = reinterpret_cast<const float4*>(W);
#pragma unroll
    for (int q = 0; q < NT / 4; ++q) {
      const float4 v = s4[q], w = w4[q];
      a = fmaf(w.x, v.x, a);
      a = fmaf(w.y, v.y, a);
      a = fmaf(w.z, v.z, a);
      a = fmaf(w.w, v.w, a);
    }
  } else {                      // 8-B aligned at RATIO = 4
    const float2* s2 = reinterpret_cast<const float2*>(src);
    const float2* w2 = reinterpret_cast<const float2*>(W);
#pragma unroll
    for (int q = 0; q < NT / 2; ++q) {
      const float2 v = s2[q], w = w2[q];
      a = fmaf(w.x, v.x, a);
      a = fmaf(w.y, v.y, a);
    }
  }
  return a;
}

// Hs[j][k] of the row (lanes over k first: rows k sit 4 banks apart), the clamped edge columns as
// their virtual columns in order (−2, −1, 0 / S − 1, S, S + 1)
template <int RATIO, int PAD>
__device__ __forceinline__ void doth_hs(const float* __restrict__ W, const float* __restrict__ Ep, int EP, int K, int S,
                                        int R, int smax, float* __restrict__ hb) {
  for (int e = threadIdx.x; e < K * S; e += blockDim.x) {
    const int k = e % K, j = e / K;
    const float* Ek = Ep + k * EP;
    const bool edge = j == 0 || j == S - 1;
    const int c0 = j == 0 ? 0 : (j == S - 1 ? S + 1 : j + 2);
    float s = doth_column<RATIO, PAD>(W, Ek, c0);
    if (edge) {
      s += doth_column<RATIO, PAD>(W, Ek, c0 + 1);
      s += doth_column<RATIO, PAD>(W, Ek, c0 + 2);
    }
    hb[(size_t)k * R * smax + j] = s;   // Hs[l][bh][k][y][j]
  }
}

template <int RMAX>
constexpr size_t doth_lds_floats(int smax, int K, int R) {
  return 64 + (size_t)((smax * K + 3) & ~3) + (size_t)K * (R + 2 * doth_pad<RMAX>() + 4);
}

template <int RMAX, int KMAX>
__global__ __launch_bounds__(256) void sel_doth_kernel(SelSmall t, const float* __restrict__ zsel, int BH, int R,
                                                       int H, int K, const long long* __restrict__ tok,
                                                       const float* __restrict__ gsel, float gscale, int smax,
                                                       float* __restrict__ Hs, float2* __restrict__ pix) {
  constexpr int PAD = doth_pad<RMAX>();
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int l = blockIdx.x / (BH * R);
  const int rem = blockIdx.x - l * (BH * R);
  const int bh = rem / R, y = rem % R;
  const int b = bh / H;
  const int S = t.s[l];
  const int ratio = R / S;
  const int EP = R + 2 * PAD + 4;       // a multiple of 4 floats: 16-B aligned row runs
  float* W = sm;                        // [64] the column filter
  float* Vs = W + 64;                   // S × K: the row's vertical pass of the selected logits
  float* Ep = Vs + ((smax * K + 3) & ~3);   // K × EP, the row's e at [PAD, PAD + R)
  const size_t RR = (size_t)R * R;
  const int x = threadIdx.x;            // blockDim.x == R
  const size_t p = (size_t)y * R + x;
  // every global load of the block first: the pixel's stats and gradient values, then the staging
  const float2 st = t.stats[l][(size_t)bh * RR + p];
  const float* gp = gsel + (size_t)b * K * RR + p;
  float gv[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < K) gv[k] = gp[(size_t)k * RR];
  unsigned selmask = 0;                 // bit k: token k selected (tok ≥ 0)
  for (int k = 0; k < K; ++k) selmask |= (tok[(size_t)b * K + k] >= 0 ? 1u : 0u) << k;
  {
    const Taps4 ty = bicubic_taps(y, S, R);
    const float* zb = zsel + t.zoff[l] + (size_t)bh * S * S * K;
    for (int e = x; e < S * K; e += blockDim.x) {
      const int j = e / K, k = e - j * K;
      float v = ty.w[0] * zb[((size_t)ty.i[0] * S + j) * K + k];
      v = fmaf(ty.w[1], zb[((size_t)ty.i[1] * S + j) * K + k], v);
      v = fmaf(ty.w[2], zb[((size_t)ty.i[2] * S + j) * K + k], v);
      v = fmaf(ty.w[3], zb[((size_t)ty.i[3] * S + j) * K + k], v);
      Vs[e] = v;
    }
  }
  for (int e = x; e < K * 2 * PAD; e += blockDim.x) {   // the zero pads
    const int k = e / (2 * PAD), q = e - k * (2 * PAD);
    Ep[k * EP + (q < PAD ? q : R + q)] = 0.0f;
  }
  const Taps4 tx = bicubic_taps(x, S, R);
  if (x < ratio) {   // phase x's weights into the filter
#pragma unroll
    for (int m = 0; m < 4; ++m) W[ratio * (3 - m) + (x + ratio / 2) % ratio] = tx.w[m];
  }
  __syncthreads();
  const float mb = __builtin_amdgcn_logf(st.y) - st.x * L2E;   // v_log_f32 = log2
  float dot = 0.0f;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k < K) {
      float e = 0.0f;
      if ((selmask >> k) & 1u) {
        float z = tx.w[0] * Vs[tx.i[0] * K + k];
        z = fmaf(tx.w[1], Vs[tx.i[1] * K + k], z);
        z = fmaf(tx.w[2], Vs[tx.i[2] * K + k], z);
        z = fmaf(tx.w[3], Vs[tx.i[3] * K + k], z);
        const float a = __builtin_amdgcn_exp2f(fmaf(z, L2E, mb));
        e = a * (gv[k] * gscale);
      }
      dot += e;
      Ep[k * EP + PAD + x] = e;
    }
  }
  pix[(size_t)l * BH * RR + (size_t)bh * RR + p] = sel_pix(mb, dot);
  __syncthreads();
  float* hb = Hs + ((size_t)l * BH + bh) * K * R * smax + (size_t)y * smax;
  if (RMAX >= 16 && ratio == 16) doth_hs<(RMAX >= 16 ? 16 : 8), PAD>(W, Ep, EP, K, S, R, smax, hb);
  else if (ratio == 8) doth_hs<8, PAD>(W, Ep, EP, K, S, R, smax, hb);
  else doth_hs<4, PAD>(W, Ep, EP, K, S, R, smax, hb);
}

// The vertical half of the sparse part's bicubicᵀ after sel_doth: es[i][j] = Σ_y A[i][y]·Hs[y][j]
// (y ascending) on the R × s rows sel_doth left in HBM.  Block = (layer, bh, k), 256 threads; LDS:
// the block's Hs rows [R][S] and the adjoint matrix as its band, Ab[i][y − y0(i)] for y in
// adj_range(i) (≤ 4·R/S + 4 entries per row; r05 held A dense, S × (R + 1), which limited the
// blocks per CU at s = 32).  Entry (i, y) belongs to output row y's thread: it zeroes its entries and
// adds its taps in order, so A is built without a barrier.
__global__ __launch_bounds__(256) void sel_adjv_kernel(SelSmall t, const float* __restrict__ Hsg, int BH, int BHK,
                                                       int smax, int R, float* __restrict__ es) {
  extern __shared__ float sh[];
  const int l = blockIdx.x / BHK;
  const int S = t.s[l];
  const int BW = 4 * (R / S) + 6;   // band width ≥ adj_range's hi − lo + 1
  float* Hs = sh;                   // R × S
  float* Ab = Hs + R * S;           // S × BW
  const size_t bk = blockIdx.x - (size_t)l * BHK;  // bh·K + k
  const float* hb = Hsg + ((size_t)l * BHK + bk) * (size_t)R * smax;   // [y][j] rows of sel_doth
  es += (size_t)l * BHK * smax * smax;
  for (int e = threadIdx.x; e < R * S; e += blockDim.x) {
    const int yy = e / S, j = e - yy * S;
    Hs[e] = hb[(size_t)yy * smax + j];
  }
  for (int y = threadIdx.x; y < R; y += blockDim.x) {
    // the rows i whose range holds y lie within [lo(y) − 2, lo(y) + 3] (lo: the first tap, before
    // clamping); the scan covers one more each side
    const int lo = bicubic_taps(y, S, R).lo;
    for (int i = max(0, lo - 3); i <= min(S - 1, lo + 4); ++i) {
      int y0, y1;
      adj_range(i, S, R, y0, y1);
      if (y >= y0 && y <= y1) Ab[i * BW + (y - y0)] = 0.0f;
    }
    const Taps4 ty = bicubic_taps(y, S, R);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      int y0, y1;
      adj_range(ty.i[m], S, R, y0, y1);
      if (y >= y0 && y <= y1) Ab[ty.i[m] * BW + (y - y0)] += ty.w[m];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < S * S; e += blockDim.x) {
    const int i = e / S, j = e - i * S;
    int y0, y1;
    adj_range(i, S, R, y0, y1);
    const float* Ai = Ab + i * BW - y0;
    float acc = 0.0f;
#pragma unroll 4
    for (int yy = y0; yy <= y1; ++yy) acc = fmaf(Ai[yy], Hs[yy * S + j], acc);
    es[bk * (size_t)S * S + e] = acc;
  }
}

// ------------------------------------------------------------------------------ sel_dense
struct SelLayers {   // up to 4 layers of the same s per launch
  const float* z[4];
  const float2* pix[4];
  const float* es[4];
  float* dz[4];
};

// output columns per band and row: 16 where R/s ≥ 8; 8 at R/s = 4 (the s = 32 layers), which keeps
// the band at 6 low-res columns and the registers under 128 (4 waves per SIMD)
template <int RATIO>
constexpr int sel_pw() { return RATIO >= 8 ? 16 : 8; }
template <int RATIO>
constexpr int sel_nc() { return lo_rel(sel_pw<RATIO>() - 1, RATIO) + 6; }   // band columns: relative −2 … lo_rel(PW−1)+3
// lanes per band: a whole wave (128-token chunks) where R/s ≥ 8; a half-wave at R/s = 4, so a block
// holds 2·R/PW bands in R/PW/2 waves (64-token chunks): the s = 32 block then needs 8 waves and
// 57 KB of LDS like the s = 16 one, two share a CU, and one launch runs both (sel_dense_pair)
template <int RATIO>
constexpr int sel_lw() { return RATIO >= 8 ? 64 : 32; }
template <int RATIO, int S>
constexpr int sel_threads() { return (S * RATIO / sel_pw<RATIO>()) * sel_lw<RATIO>(); }
template <int RATIO, int S>
constexpr int sel_lds_m() { return (S * RATIO / sel_pw<RATIO>()) * sel_nc<RATIO>() * sel_lw<RATIO>(); }   // f2
template <int RATIO, int S>
constexpr int sel_lds_z() { return 4 * (S + 4) * sel_lw<RATIO>(); }                                       // f2

// One job = (layer l, head bh, token chunk of 2·LW); NB = R/PW bands of LW lanes, band bw owns
// output columns [PW·bw, PW·bw + PW) of every row, lanes own token pairs.  The 4 low-res z rows
// the current output rows interpolate sit in an LDS ring Z[slot][column][lane] shared by all bands
// (bands overlap, so each column is loaded once per block); the next row is fetched into registers
// at the start of a phase and stored into the retired slot behind the emit's first barrier.  acc
// (the vertical adjoint of the 4 rows) and the per-row V / Hs stay in registers.
template <int RATIO, int S>
__device__ __forceinline__ void sel_dense_body(const SelLayers& sl, int BH, int H, int N, int K,
                                               const long long* __restrict__ tok, int nchunk, int job, f2* M, f2* Z,
                                               int tid0) {
  constexpr int PW = sel_pw<RATIO>();
  constexpr int LW = sel_lw<RATIO>();
  constexpr int R = S * RATIO;
  constexpr int NB = R / PW;                      // bands
  constexpr int CS = PW / RATIO;                  // band step in low-res columns
  constexpr int NC = sel_nc<RATIO>();
  constexpr int CPT = (S + NB - 1) / NB;          // ring columns each thread fetches per row
  constexpr int TPC = 2 * LW;                     // tokens per chunk
  static_assert(R % PW == 0 && PW % RATIO == 0, "band geometry");
  const int chunk = job % nchunk;
  const int bh = (job / nchunk) % BH;
  const int l = job / (nchunk * BH);
  const int b = bh / H;
  const int tid = tid0, lane = tid & (LW - 1);   // the thread's index within its job's threads
  // band of this thread: the wave (uniform) or, at LW = 32, the wave's half
  const int bw = LW == WAVE ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid / LW;
  const int n0 = chunk * TPC + 2 * lane;
  const int nl = min(n0, N - 2);                   // clamped load position (N even)
  const float* zl = sl.z[l] + (size_t)bh * S * S * N;
  const float2* pixl = sl.pix[l] + (size_t)bh * R * R;
  float* dzl = sl.dz[l] + (size_t)bh * S * S * N;
  const float* esl = sl.es[l] ? sl.es[l] + (size_t)bh * K * S * S : nullptr;
  // the selected rows this lane's token pair (n0, n0 + 1) carries (bit k: tok_k; duplicates add)
  unsigned mx = 0u, my = 0u;
  for (int k = 0; k < K; ++k) {
    const long long t = tok[(size_t)b * K + k];
    if (t == n0) mx |= 1u << k;
    if (t == n0 + 1) my |= 1u << k;
  }

  // tap weights of the RATIO phases (identical for rows and columns): lane u < RATIO computes
  // phase u's taps exactly as the forward did, then every lane reads them as uniform values
  float wt[RATIO][4];
  {
    const int wl = tid & 63;
    const Taps4 t = bicubic_taps(wl < RATIO ? wl : 0, S, R);
#pragma unroll
    for (int u = 0; u < RATIO; ++u)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        wt[u][m] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t.w[m]), u));
  }
  // ring rows carry two virtual columns each side (−2, −1 = column 0; S, S + 1 = column S − 1, as
  // torch's clamped taps), so band slot c of band bw is ring column bw·CS + c: no clamp per read
  constexpr int SP = S + 4;
  auto slot = [](int r) { return (r + 4) & 3; };   // virtual rows ≥ −2
  f2 pre[CPT];
  auto fetch = [&](int r) {   // z_low row r (clamped): this thread's ring columns, its lane's token pair
    const int rr = min(max(r, 0), S - 1);
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int col = bw + k * NB;
      if (col < S) pre[k] = *reinterpret_cast<const f2*>(zl + ((size_t)rr * S + col) * N + nl);
    }
  };
  auto stash = [&](int r) {
    f2* zs = Z + slot(r) * SP * LW;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int col = bw + k * NB;
      if (col < S) {
        zs[(col + 2) * LW + lane] = pre[k];
        if (col == 0) { zs[lane] = pre[k]; zs[LW + lane] = pre[k]; }
        if (col == S - 1) { zs[(S + 2) * LW + lane] = pre[k]; zs[(S + 3) * LW + lane] = pre[k]; }
      }
    }
  };
#pragma unroll 1
  for (int r = -2; r <= 1; ++r) {
    fetch(r);
    stash(r);
  }
  __syncthreads();

  f2 acc[4][NC];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[k][c] = (f2)0.0f;
  const f2 l2e = (f2)L2E;

  // low-res row r complete: merge the bands, add es at the selected tokens, store; then the
  // fetched row `next` goes into the retired slot (every band is past its reads of it)
  auto emit = [&](int r, const f2 (&v)[NC], int next) {
#pragma unroll
    for (int c = 0; c < NC; ++c) M[(bw * NC + c) * LW + lane] = v[c];
    __syncthreads();
    const int n = chunk * TPC + 2 * lane;
    for (int j = bw; j < S; j += NB) {   // a band per low-res column (uniform j per band)
      f2 s = (f2)0.0f;
      if (j == 0 || j == S - 1) {   // clamped edge columns: every (band, column) folding into j, band order
        for (int w2 = 0; w2 < NB; ++w2)
          for (int c = 0; c < NC; ++c)
            if (min(max(w2 * CS + c - 2, 0), S - 1) == j) s += M[(w2 * NC + c) * LW + lane];
      } else {                      // interior: one column per band, c = j + 2 − w2·CS (band order)
        const int wlo = max(0, (j + 2 - NC + CS) / CS), whi = min(NB - 1, (j + 2) / CS);
        for (int w2 = wlo; w2 <= whi; ++w2) s += M[(w2 * NC + j + 2 - w2 * CS) * LW + lane];
      }
      if (n < N) {
        if (esl) {   // the sparse part es at the selected tokens, k order
          for (unsigned m = mx; m; m &= m - 1) s.x += esl[((size_t)__builtin_ctz(m) * S + r) * S + j];   // k order
          for (unsigned m = my; m; m &= m - 1) s.y += esl[((size_t)__builtin_ctz(m) * S + r) * S + j];
        }
        *reinterpret_cast<f2*>(dzl + ((size_t)r * S + j) * N + n) = s;
      }
    }
    if (next <= S + 1) stash(next);
    __syncthreads();
  };

  // phases: lo = first tap row of the output rows y = RATIO·(lo + 1) + RATIO/2 + v, v = 0..RATIO−1
#pragma unroll 1
  for (int lo = -2; lo <= S - 2; ++lo) {
    const bool more = lo + 1 <= S - 2;             // the next phase needs row lo + 4
    if (more) fetch(lo + 4);
    const f2* z0 = Z + slot(lo) * SP * LW + bw * CS * LW + lane;
    const f2* z1 = Z + slot(lo + 1) * SP * LW + bw * CS * LW + lane;
    const f2* z2 = Z + slot(lo + 2) * SP * LW + bw * CS * LW + lane;
    const f2* z3 = Z + slot(lo + 3) * SP * LW + bw * CS * LW + lane;
#pragma unroll
    for (int v = 0; v < RATIO; ++v) {
      const int y = RATIO * (lo + 1) + RATIO / 2 + v;
      if (y < 0 || y >= R) continue;   // the first and last phases have RATIO/2 rows
      const int u = (RATIO / 2 + v) % RATIO;   // row phase (compile-time)
      f2 V[NC], Hs[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int o = c * LW;
        f2 t = z0[o] * wt[u][0];
        t = __builtin_elementwise_fma(z1[o], (f2)wt[u][1], t);
        t = __builtin_elementwise_fma(z2[o], (f2)wt[u][2], t);
        t = __builtin_elementwise_fma(z3[o], (f2)wt[u][3], t);
        V[c] = t;
        Hs[c] = (f2)0.0f;
      }
      const float2* pp = pixl + (size_t)y * R + bw * PW;
#pragma unroll
      for (int t = 0; t < PW; ++t) {
        const int ut = t % RATIO;
        const int c0 = lo_rel(t, RATIO) + 2;                             // band slot of the first tap
        // (mb, d), uniform per band: a scalar load where the band is the wave (read-only here)
        float2 pd;
        if constexpr (LW == WAVE && SKP_SEL_DFOLD) {
          using cu64 = __attribute__((address_space(4))) const unsigned long long;
          pd = __builtin_bit_cast(float2, reinterpret_cast<cu64*>(reinterpret_cast<uintptr_t>(pp))[t]);
        } else {
          pd = pp[t];
        }
        f2 zv = V[c0] * wt[ut][0];
        zv = __builtin_elementwise_fma(V[c0 + 1], (f2)wt[ut][1], zv);
        zv = __builtin_elementwise_fma(V[c0 + 2], (f2)wt[ut][2], zv);
        zv = __builtin_elementwise_fma(V[c0 + 3], (f2)wt[ut][3], zv);
        f2 ex = __builtin_elementwise_fma(zv, l2e, (f2)pd.x);
        ex.x = __builtin_amdgcn_exp2f(ex.x);
        ex.y = __builtin_amdgcn_exp2f(ex.y);
        float w4[4] = {wt[ut][0], wt[ut][1], wt[ut][2], wt[ut][3]};
#if SKP_SEL_DFOLD
        if constexpr (LW == WAVE) {
          // ex = a·|d| (sel_pix); d's sign (uniform: one band per wave) flips the tap weights'
          // sign bits in SGPRs — no VALU
          const unsigned sg = __builtin_bit_cast(unsigned, pd.y) & 0x80000000u;
#pragma unroll
          for (int m = 0; m < 4; ++m) w4[m] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, w4[m]) ^ sg);
        } else {   // two bands per wave: the sign as a packed multiply, as without the fold
          ex *= (f2)__builtin_copysignf(1.0f, pd.y);
        }
#else
        ex *= pd.y;
#endif
        Hs[c0] = __builtin_elementwise_fma(ex, (f2)w4[0], Hs[c0]);
        Hs[c0 + 1] = __builtin_elementwise_fma(ex, (f2)w4[1], Hs[c0 + 1]);
        Hs[c0 + 2] = __builtin_elementwise_fma(ex, (f2)w4[2], Hs[c0 + 2]);
        Hs[c0 + 3] = __builtin_elementwise_fma(ex, (f2)w4[3], Hs[c0 + 3]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[k][c] = __builtin_elementwise_fma(Hs[c], (f2)wt[u][k], acc[k][c]);
    }
    // virtual row lo is complete
    if (lo < 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[1][c] += acc[0][c];   // rows −2, −1 clamp to row 0 (next slot)
      __syncthreads();                                        // every band past its reads of slot(lo)
      if (more) stash(lo + 4);
      __syncthreads();
    } else {
      emit(lo, acc[0], more ? lo + 4 : S + 2);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      acc[0][c] = acc[1][c]; acc[1][c] = acc[2][c]; acc[2][c] = acc[3][c]; acc[3][c] = (f2)0.0f;
    }
  }
  // the window now holds virtual rows S−1, S, S+1, S+2: all clamp to row S−1
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[0][c] = (acc[0][c] + acc[1][c]) + (acc[2][c] + acc[3][c]);
  emit(S - 1, acc[0], S + 2);
}

// XCD-major job order: XCD x walks a contiguous job range, so a head's token chunks share one L2
// (its z_low slab)
__device__ __forceinline__ int xcd_job(int njobs) {
  const int per = (njobs + 7) / 8;
  return (blockIdx.x & 7) * per + (blockIdx.x >> 3);
}

template <int RATIO, int S>
__global__ __launch_bounds__((sel_threads<RATIO, S>()))
void sel_dense_kernel(SelLayers sl, int BH, int H, int N, int K, const long long* __restrict__ tok, int nchunk,
                      int njobs) {
  __shared__ __attribute__((aligned(16))) f2 M[sel_lds_m<RATIO, S>()];   // band partials of one low-res row
  __shared__ __attribute__((aligned(16))) f2 Z[sel_lds_z<RATIO, S>()];   // ring of 4 low-res z rows
  const int job = xcd_job(njobs);
  if (job >= njobs) return;
  sel_dense_body<RATIO, S>(sl, BH, H, N, K, tok, nchunk, job, M, Z, threadIdx.x);
}

// Two layer classes (e.g. SD-1.5's s = 16 layers and its s = 32 layer at R = 128) in ONE grid of
// equal-size blocks: per XCD, its share of class A's blocks first, then its share of class B's, so
// the class-B blocks fill the slots class A's last round leaves idle (two launches left half of the
// CUs idle in the s = 16 launch's last round and ran the s = 32 launch alone).  (r05 measured a
// 16-wave form with two class-A jobs per block side by side — bit-identical, 5% slower,
// profiles/r05zf_sel_dual_ab.txt — removed in r06.)
template <int RA, int SA, int RB, int SB>
__global__ __launch_bounds__((sel_threads<RB, SB>()))
void sel_dense_pair_kernel(SelLayers sa, int nca, int ja, SelLayers sb, int ncb, int jb, int BH, int H, int N, int K,
                           const long long* __restrict__ tok) {
  static_assert(sel_threads<RA, SA>() == sel_threads<RB, SB>(), "the two classes' blocks must be equal");
  constexpr int MA = sel_lds_m<RA, SA>(), MB = sel_lds_m<RB, SB>();
  constexpr int ZA = sel_lds_z<RA, SA>(), ZB = sel_lds_z<RB, SB>();
  constexpr int LA = MA + ZA, LB = MB + ZB;
  __shared__ __attribute__((aligned(16))) f2 lds[LA > LB ? LA : LB];
  const int pa = (ja + 7) / 8, pb = (jb + 7) / 8;   // per-XCD shares
  const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
  if (k < pa) {
    const int job = xcd * pa + k;
    if (job < ja) sel_dense_body<RA, SA>(sa, BH, H, N, K, tok, nca, job, lds, lds + MA, threadIdx.x);
  } else {
    const int job = xcd * pb + (k - pa);
    if (job < jb) sel_dense_body<RB, SB>(sb, BH, H, N, K, tok, ncb, job, lds, lds + MB, threadIdx.x);
  }
}

template <int RATIO, int S>
void launch_dense(const SelLayers& sl, int nl, int BH, int H, int N, int K, const long long* tok, hipStream_t st) {
  const int nchunk = (N + 2 * sel_lw<RATIO>() - 1) / (2 * sel_lw<RATIO>());
  const int njobs = nl * BH * nchunk;
  const int grid = 8 * ((njobs + 7) / 8);
  hipLaunchKernelGGL((sel_dense_kernel<RATIO, S>), dim3(grid), dim3(sel_threads<RATIO, S>()), 0, st, sl, BH, H, N, K,
                     tok, nchunk, njobs);
}

template <int RA, int SA, int RB, int SB>
void launch_dense_pair(const SelLayers& sa, int na, const SelLayers& sb, int nb, int BH, int H, int N, int K,
                       const long long* tok, hipStream_t st) {
  const int nca = (N + 2 * sel_lw<RA / SA>() - 1) / (2 * sel_lw<RA / SA>());
  const int ncb = (N + 2 * sel_lw<RB / SB>() - 1) / (2 * sel_lw<RB / SB>());
  const int ja = na * BH * nca, jb = nb * BH * ncb;
  const int grid = 8 * ((ja + 7) / 8 + (jb + 7) / 8);
  hipLaunchKernelGGL((sel_dense_pair_kernel<RA / SA, SA, RB / SB, SB>), dim3(grid), dim3(sel_threads<RB / SB, SB>()), 0,
                     st, sa, nca, ja, sb, ncb, jb, BH, H, N, K, tok);
}

#ifndef SKP_SEL_PAIR
#define SKP_SEL_PAIR 1   // 0: one sel_dense launch per layer size (A/B build)
#endif

// (R, S) pairs with a compiled sel_dense kernel
bool dense_launch(int R, int S, const SelLayers& sl, int nl, int BH, int H, int N, int K, const long long* tok,
                  hipStream_t st) {
#define SKP_SEL_CASE(RR, SS)                                               \
  if (R == RR && S == SS) {                                               \
    launch_dense<RR / SS, SS>(sl, nl, BH, H, N, K, tok, st);               \
    return true;                                                          \
  }
  SKP_SEL_CASE(128, 16)
  SKP_SEL_CASE(128, 32)
  SKP_SEL_CASE(128, 8)
  SKP_SEL_CASE(64, 16)
  SKP_SEL_CASE(64, 8)
  SKP_SEL_CASE(64, 4)
  SKP_SEL_CASE(32, 8)
  SKP_SEL_CASE(32, 4)
#undef SKP_SEL_CASE
  return false;
}

// the SD-1.5 capture layers at R = 128 (s = 16 ×3 and s = 32) as one sel_dense_pair launch
bool dense_pair_launch(int R, int SA, const SelLayers& sa, int na, int SB, const SelLayers& sb, int nb, int BH, int H,
                       int N, int K, const long long* tok, hipStream_t st) {
#if SKP_SEL_PAIR
  if (R == 128 && SA == 16 && SB == 32) {
    launch_dense_pair<128, 16, 128, 32>(sa, na, sb, nb, BH, H, N, K, tok, st);
    return true;
  }
  if (R == 128 && SA == 32 && SB == 16) {
    launch_dense_pair<128, 16, 128, 32>(sb, nb, sa, na, BH, H, N, K, tok, st);
    return true;
  }
#endif
  return false;
}

bool dense_supported(int R, int S) {
  const int pairs[][2] = {{128, 16}, {128, 32}, {128, 8}, {64, 16}, {64, 8}, {64, 4}, {32, 8}, {32, 4}};
  for (auto& p : pairs)
    if (p[0] == R && p[1] == S) return true;
  return false;
}

// dense gradient from the sparse one (fallback): g[b][tok_k][p] = Σ_k gsel[b][k][p] (k order)
__global__ void sel_scatter_kernel(const long long* __restrict__ tok, const float* __restrict__ gsel, int B, int K,
                                   int N, long long RR, float* __restrict__ g) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // (b, p)
  if (e >= (long long)B * RR) return;
  const int b = (int)(e / RR);
  const long long p = e % RR;
  for (int k = 0; k < K; ++k) {
    const long long t = tok[(long long)b * K + k];
    if (t >= 0 && t < N) g[((long long)b * N + t) * RR + p] += gsel[((long long)b * K + k) * RR + p];
  }
}

template <int RMAX>
void launch_doth(const SelSmall& t, int L, int BH, int R, int H, int K, int smax, const long long* tok,
                 const float* gsel, float gscale, const float* zsel, float* hs, float2* pix, hipStream_t st) {
  const size_t lds = doth_lds_floats<RMAX>(smax, K, R) * sizeof(float);
  if (K <= 16)   // the pixel's gradient values are held in registers: 16 or SEL_MAXK of them
    hipLaunchKernelGGL((sel_doth_kernel<RMAX, 16>), dim3((unsigned)(L * BH * R)), dim3(R), lds, st, t, zsel, BH, R, H, K,
                       tok, gsel, gscale, smax, hs, pix);
  else
    hipLaunchKernelGGL((sel_doth_kernel<RMAX, SEL_MAXK>), dim3((unsigned)(L * BH * R)), dim3(R), lds, st, t, zsel, BH, R,
                       H, K, tok, gsel, gscale, smax, hs, pix);
}

struct SelWs {   // workspace carve-up (floats)
  size_t zsel, hs, pix, es, total;
};
SelWs sel_ws(const int* sizes, int L, int B, int H, int R, int K) {
  SelWs w{};
  size_t smax = 1;
  for (int l = 0; l < L; ++l) smax = std::max(smax, (size_t)sizes[l]);
  const size_t smax2 = smax * smax;
  const size_t BH = (size_t)B * H, RR = (size_t)R * R;
  size_t zs = 0;
  for (int l = 0; l < L; ++l) zs += BH * (size_t)sizes[l] * sizes[l] * K;
  w.zsel = 0;
  w.hs = w.zsel + ((zs + 3) & ~(size_t)3);                // sel_doth's Hs rows [l][bh][k][R][smax]
  w.pix = w.hs + (((size_t)L * BH * K * R * smax + 3) & ~(size_t)3);
  w.es = w.pix + (size_t)L * BH * RR * 2;
  w.total = w.es + (size_t)L * BH * K * smax2;
  return w;
}

// Per-phase timing of the fast path (skp_sel_bwd_timing*): when enabled, each call records 5 events
// on its stream — before sel_gather, after sel_gather, after sel_doth, after sel_adjv, after
// sel_dense — into a pool read back by skp_sel_bwd_timing_read.  A call's slot counts only once its
// last event is recorded, so a call that returns early leaves no half-recorded slot behind.  Off by
// default (no events recorded); one caller thread at a time (the bench).
struct SelTiming {
  bool on = false;
  int n = 0;                       // complete calls recorded since the last read
  std::vector<hipEvent_t> ev;      // 5 per call
};
SelTiming& sel_timing() {
  static SelTiming t;
  return t;
}
constexpr int SEL_TIMING_MAX_CALLS = 256;
hipEvent_t* sel_timing_slot() {   // the next call's 5 events (committed by sel_timing_commit), or null
  SelTiming& t = sel_timing();
  if (!t.on || t.n >= SEL_TIMING_MAX_CALLS) return nullptr;
  while ((int)t.ev.size() < 5 * (t.n + 1)) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    t.ev.push_back(e);
  }
  return &t.ev[5 * t.n];
}
void sel_timing_commit() { ++sel_timing().n; }

// (R, s) pairs of the fast path: a compiled sel_dense kernel, and R/s ∈ {4, 8, 16} — the column
// filters sel_doth instantiates (its W table holds 4·RATIO ≤ 64 taps)
bool fast_path(const int* sizes, int L, int R, int N) {
  if (N % 2 != 0 || N < 2 || R > 256) return false;
  for (int l = 0; l < L; ++l) {
    if (!dense_supported(R, sizes[l])) return false;
    const int ratio = R / sizes[l];
    if (R % sizes[l] != 0 || (ratio != 4 && ratio != 8 && ratio != 16)) return false;
  }
  return true;
}

}  // namespace

extern "C" long long skp_capture_maps_bwd_sel_workspace(const int* sizes, int L, int B, int H, int N, int R, int K) {
  if (!sizes || L <= 0 || L > SKP_MAX_LAYERS || B <= 0 || H <= 0 || N <= 0 || R <= 0 || K <= 0) return -1;
  int smax = 1;
  for (int l = 0; l < L; ++l) smax = std::max(smax, sizes[l]);
  if (fast_path(sizes, L, R, N)) return (long long)sel_ws(sizes, L, B, H, R, K).total;
  // fallback: the dense (B, N, R²) gradient + skp_capture_maps_bwd's workspace
  const long long RR = (long long)R * R;
  return (long long)B * N * RR + (long long)B * RR * N + (long long)B * H * R * smax * N + 4;
}

extern "C" int skp_capture_maps_bwd_sel(const float* const* z_low, const int* sizes, int L, int B, int H, int N, int R,
                                        const long long* sel_tok, int K, const float* gsel, float gscale,
                                        const float* const* stats, float* const* dz_low, float* workspace,
                                        void* stream) {
  SKP_CHECK_ARG(z_low && sizes && sel_tok && gsel && stats && dz_low && workspace, "null pointer");
  SKP_CHECK_ARG(L > 0 && L <= SKP_MAX_LAYERS, "L out of range");
  SKP_CHECK_ARG(B > 0 && H > 0 && N > 0 && R > 0, "non-positive shape");
  SKP_CHECK_ARG(R % 4 == 0, "R must be a multiple of 4");
  SKP_CHECK_ARG(K > 0 && K <= SEL_MAXK, "K must be in [1, 32]");
  SKP_CHECK_ARG(N % 4 == 0 && N <= 1024, "N must be a multiple of 4, at most 1024");
  SKP_CHECK_ARG((long long)B * H <= 65535 && (long long)B * H * R * R < (1LL << 31), "shape too large");
  SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "workspace must be 16-B aligned");
  for (int l = 0; l < L; ++l) {
    SKP_CHECK_ARG(z_low[l] && dz_low[l] && stats[l], "null layer pointer");
    SKP_CHECK_ARG(sizes[l] > 0 && sizes[l] <= R, "layer size must be in [1, R]");
    SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(z_low[l]) & 15) == 0 && (reinterpret_cast<uintptr_t>(dz_low[l]) & 15) == 0,
                  "z_low / dz_low pointers must be 16-B aligned");
  }
  hipStream_t st = as_stream(stream);
  const int BH = B * H;
  const size_t RR = (size_t)R * R;
  if (!fast_path(sizes, L, R, N)) {
    // no compiled kernel for this (R, s): scatter into a dense gradient, then the dense backward
    float* g = workspace;
    SKP_CHECK_ARG(hipMemsetAsync(g, 0, (size_t)B * N * RR * sizeof(float), st) == hipSuccess, "memset failed");
    hipLaunchKernelGGL(sel_scatter_kernel, dim3((unsigned)(((size_t)B * RR + 255) / 256)), dim3(256), 0, st, sel_tok,
                       gsel, B, K, N, (long long)RR, g);
    SKP_LAUNCH_CHECK();
    float* rest = workspace + (((size_t)B * N * RR + 3) & ~(size_t)3);
    return skp_capture_maps_bwd(z_low, sizes, L, B, H, N, R, g, gscale, stats, dz_low, rest, stream);
  }
  const SelWs wsz = sel_ws(sizes, L, B, H, R, K);
  float* zsel = workspace + wsz.zsel;
  float* hs = workspace + wsz.hs;
  float2* pix = reinterpret_cast<float2*>(workspace + wsz.pix);
  float* es = workspace + wsz.es;
  int smax = 1, rmax = 1;
  for (int l = 0; l < L; ++l) {
    smax = std::max(smax, sizes[l]);
    rmax = std::max(rmax, R / sizes[l]);
  }
  SelSmall t{};
  t.zoff[0] = 0;
  for (int l = 0; l < L; ++l) {
    t.z[l] = z_low[l];
    t.stats[l] = reinterpret_cast<const float2*>(stats[l]);
    t.s[l] = sizes[l];
    t.zoff[l + 1] = t.zoff[l] + (long long)BH * sizes[l] * sizes[l] * K;
  }
  hipEvent_t* tev = sel_timing_slot();
  if (tev) (void)hipEventRecord(tev[0], st);
  hipLaunchKernelGGL(sel_gather_kernel, dim3((unsigned)((t.zoff[L] + 255) / 256)), dim3(256), 0, st, t, L, BH, N, H,
                     sel_tok, K, zsel);
  SKP_LAUNCH_CHECK();
  if (tev) (void)hipEventRecord(tev[1], st);
  // sel_doth: per (layer, bh, row) a_k, e_k = a_k·g_k and dot, with the horizontal half of the
  // sparse part's bicubicᵀ applied in LDS (Hs rows; the R² e rows never reach HBM)
  if (rmax <= 8) launch_doth<8>(t, L, BH, R, H, K, smax, sel_tok, gsel, gscale, zsel, hs, pix, st);
  else launch_doth<16>(t, L, BH, R, H, K, smax, sel_tok, gsel, gscale, zsel, hs, pix, st);
  SKP_LAUNCH_CHECK();
  if (tev) (void)hipEventRecord(tev[2], st);
  // sel_adjv: the vertical half → es[l][bh][k] (s × s per selected row)
  hipLaunchKernelGGL(sel_adjv_kernel, dim3((unsigned)(L * BH * K)), dim3(256),
                     (size_t)(R * smax + 4 * R + 6 * smax) * sizeof(float), st, t, hs, BH, BH * K, smax, R, es);
  SKP_LAUNCH_CHECK();
  if (tev) (void)hipEventRecord(tev[3], st);
  // the dense part: layers of equal s share a class (up to 4 per launch); two classes that have
  // a paired kernel (SD-1.5: s = 16 and 32 at R = 128) run as one launch
  SelLayers cls[SKP_MAX_LAYERS];
  int cls_s[SKP_MAX_LAYERS], cls_n[SKP_MAX_LAYERS], ncls = 0;
  bool done[SKP_MAX_LAYERS] = {};
  for (int l = 0; l < L; ++l) {
    if (done[l]) continue;
    SelLayers sl{};
    int nl = 0;
    for (int m = l; m < L && nl < 4; ++m) {
      if (done[m] || sizes[m] != sizes[l]) continue;
      sl.z[nl] = z_low[m];
      sl.pix[nl] = pix + (size_t)m * BH * RR;
      sl.es[nl] = es + (size_t)m * BH * K * smax * smax;
      sl.dz[nl] = dz_low[m];
      done[m] = true;
      ++nl;
    }
    cls[ncls] = sl;
    cls_s[ncls] = sizes[l];
    cls_n[ncls] = nl;
    ++ncls;
  }
  if (!(ncls == 2 && dense_pair_launch(R, cls_s[0], cls[0], cls_n[0], cls_s[1], cls[1], cls_n[1], BH, H, N, K, sel_tok,
                                       st))) {
    for (int c = 0; c < ncls; ++c)
      SKP_CHECK_ARG(dense_launch(R, cls_s[c], cls[c], cls_n[c], BH, H, N, K, sel_tok, st),
                    "internal: no sel_dense kernel for this shape");
  }
  SKP_LAUNCH_CHECK();
  if (tev) {
    (void)hipEventRecord(tev[4], st);
    sel_timing_commit();
  }
  return SKP_OK;
}

extern "C" int skp_sel_bwd_timing(int enable) {
  SelTiming& t = sel_timing();
  t.on = enable != 0;
  t.n = 0;
  return SKP_OK;
}

extern "C" int skp_sel_bwd_timing_read(double* ms, int* calls) {
  SKP_CHECK_ARG(ms && calls, "null pointer");
  SelTiming& t = sel_timing();
  for (int k = 0; k < 4; ++k) ms[k] = 0.0;
  for (int c = 0; c < t.n; ++c) {
    hipEvent_t* e = &t.ev[5 * c];
    SKP_CHECK_ARG(hipEventSynchronize(e[4]) == hipSuccess, "event sync failed");
    for (int k = 0; k < 4; ++k) {
      float v = 0.0f;
      SKP_CHECK_ARG(hipEventElapsedTime(&v, e[k], e[k + 1]) == hipSuccess, "elapsed time failed");
      ms[k] += v;
    }
  }
  *calls = t.n;
  t.n = 0;
  return SKP_OK;
}
