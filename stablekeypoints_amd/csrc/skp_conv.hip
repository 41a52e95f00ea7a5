// 3×3 / stride-1 / pad-1 convolution of the frozen SD VAE and UNet as Winograd F(4×4, 3×3) on
// the gfx950 fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulate).
//
// The hot path encodes every image and its warp with the VAE each optimiser step
// (reference ptp_utils.py:289-304 image2latent, called from optimize.py:173-180) and runs the
// UNet forward and its input-gradient backward; their 3×3 convolutions are ≈60% of the step.
// gfx950 has no reduced-precision f32 MFMA (no xf32), so the f32 matrix rate (157 TF/s, the
// same as the vector rate) is the ceiling for a direct convolution.  F(4×4, 3×3) computes a
// 4×4 output tile from a 6×6 input tile with 36 multiplies per (input, output) channel pair
// instead of 144: a 4× cut of the matrix-core work, paid for with transforms on the VALU.
//
// Interpolation points (0, 1, -1, 1/2, -2, ∞): all input/output transform coefficients are
// dyadic (exact in fp32) and the fp32 error is ≈3× a direct sequential fp32 sum (the classic
// (0, ±1, ±2, ∞) points give ≈6×); tests/test_gpu_conv.py bounds it against fp64.
//
//   V = Bᵀ d B   (6×6 input tile d of one channel, on the VALU, into LDS)
//   U = G g Gᵀ   (6×6 per (out, in) channel pair; precomputed once per frozen weight, fp64)
//   M_p = Σ_c U_p[c][k] · V_p[c][t]   for each of the 36 positions p: 36 GEMMs on MFMA
//   Y = Aᵀ M A   (4×4 output tile, in registers, + bias + residual in the same epilogue)
//
// Workgroup: 64 output tiles × 32 output channels, 8 waves (two per SIMD); wave w owns tiles
// 16(w&3)..+15 × channels 16(w>>2)..+15 as one 16×16 MFMA block per position, so each lane
// ends holding all 36 positions of 4 tiles × 1 channel (144 accumulator registers) and runs
// the output transform without any data exchange.  Input channels are walked four at a time;
// the stage pipeline keeps no loads in registers (LDS-DMA, buffer_load … lds):
//   waves 0-3 (wave w = channel w of a stage, lane = tile): transform the raw 6×6 patches of
//     stage s+1 (already in LDS) into V[s+1], then DMA stage s+2's raw patches into the same
//     per-wave LDS area, then their MFMAs on stage s;
//   waves 4-7: DMA stage s+1's U slice into U[s+1], then their MFMAs on stage s;
// one barrier per stage.  The two waves of a SIMD are one of each kind, so one's transform
// runs under the other's MFMAs.  The workgroup → (tile block, channel block) map keeps the
// work that shares operands on one XCD's L2: tile-major when the whole U fits an L2 slice
// (every channel block of a tile block back to back), channel-block-major otherwise.
//
// The backward of the same convolution w.r.t. its input is the same correlation of dy with
// the 180°-rotated, in/out-transposed kernel: skp_wino_weights(flip=1) builds that U.
#include <cstdlib>

#include "skp_common.h"

using namespace skp;

// Timing-probe builds only (tools/build_variant.sh, e.g. EXTRA=-DSKP_WINO2_DEBUG=8); the shipped
// library is built with 0.  wino_f4_kernel: 1 drop x loads, 2 drop U loads, 4 skip transforms,
// 8 skip MFMAs.  wino2_kernel: 1 skip transforms, 2 skip MFMAs, 4 skip input DMA, 8 skip weight
// DMA, 16 skip the stage loop, 32 skip the epilogue, 64 skip its global stores.
#ifndef SKP_WINO_DEBUG
#define SKP_WINO_DEBUG 0
#endif
#ifndef SKP_WINO2_DEBUG
#define SKP_WINO2_DEBUG 0
#endif

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kMT = 64;                       // output tiles per workgroup
constexpr int kNC = 32;                       // output channels per workgroup
constexpr int kCK = 4;                        // input channels per LDS stage (= MFMA k)
constexpr int kP = 36;                        // transform positions (6×6)
constexpr int kThreads = 512;                 // 8 waves, two per SIMD
// V stage: kCK · MT · kP floats (9216 at MT = 64)
constexpr int kUs = kCK * kNC * kP;           // floats per U stage  (4608)
constexpr int kUChunks = kUs * 4 / 1024;      // 1-KB DMA chunks per U stage (18)
constexpr int kRawRow = 64 * 16 + 64 * 4 + 64 * 4;   // bytes per patch row per wave: middle, left, right
constexpr int kRawWave = 6 * kRawRow;         // 9216 B: one wave's 64 raw patches
// LDS: V 2 × 36 KB + U 2 × 18 KB + raw patches 36 KB = 147.5 KB (static)

static_assert(kMT == 64 && kCK == 4, "wave w of 0..3 = stage channel w, lane = tile");
static_assert(kUs * 4 % 1024 == 0, "U stage in whole 1-KB chunks");

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// y = Bᵀ x for the points (0, 1, -1, 1/2, -2, ∞)
__device__ __forceinline__ void bt6(float a0, float a1, float a2, float a3, float a4, float a5, float* y, int s) {
  y[0 * s] = a0 - 1.5f * a1 - 2.0f * a2 + 1.5f * a3 + a4;
  y[1 * s] = -a1 + 0.5f * a2 + 2.5f * a3 + a4;
  y[2 * s] = a1 - 2.5f * a2 + 0.5f * a3 + a4;
  y[3 * s] = -2.0f * a1 - a2 + 2.0f * a3 + a4;
  y[4 * s] = 0.5f * a1 - a2 - 0.5f * a3 + a4;
  y[5 * s] = a1 - 1.5f * a2 - 2.0f * a3 + 1.5f * a4 + a5;
}

// y = Aᵀ m (4 outputs from 6 positions)
__device__ __forceinline__ void at6(float m0, float m1, float m2, float m3, float m4, float m5, float* y, int s) {
  const float p = m1 + m2, q = m1 - m2;
  y[0 * s] = m0 + p + m3 + m4;
  y[1 * s] = q + 0.5f * m3 - 2.0f * m4;
  y[2 * s] = p + 0.25f * m3 + 4.0f * m4;
  y[3 * s] = q + 0.125f * m3 - 8.0f * m4 + m5;
}

// V = Bᵀ d B, d and v row-major 6×6
__device__ __forceinline__ void input_transform(const float* d, float* v) {
  float t[36];
#pragma unroll
  for (int c = 0; c < 6; ++c) bt6(d[c], d[6 + c], d[12 + c], d[18 + c], d[24 + c], d[30 + c], t + c, 6);
#pragma unroll
  for (int r = 0; r < 6; ++r) bt6(t[6 * r], t[6 * r + 1], t[6 * r + 2], t[6 * r + 3], t[6 * r + 4], t[6 * r + 5], v + 6 * r, 1);
}

// Y = Aᵀ M A, m row-major 6×6, y row-major 4×4
__device__ __forceinline__ void output_transform(const float* m, float* y) {
  float s[24];
#pragma unroll
  for (int c = 0; c < 6; ++c) at6(m[c], m[6 + c], m[12 + c], m[18 + c], m[24 + c], m[30 + c], s + c, 6);
#pragma unroll
  for (int r = 0; r < 4; ++r) at6(s[6 * r], s[6 * r + 1], s[6 * r + 2], s[6 * r + 3], s[6 * r + 4], s[6 * r + 5], y + 4 * r, 1);
}

// DMA one wave's 64 raw 6×6 patches (lane = tile) of one channel plane into its LDS area:
// per patch row, the aligned middle four columns (16 B), the left and the right column (4 B
// each), each as one buffer_load … lds with lane-linear destinations.  Source rows are clamped
// into the plane and the left/right columns into the tensor; the zero padding is applied at
// transform time from the per-lane mask (bits 0..5 row inside, 6 left, 7 right column).
struct PatchAddr {
  unsigned row[6];   // byte offset of (row y0-1+r clamped, col x0) from the stage's channel-0 plane
  unsigned dl;       // 4 when the left column exists (x0 > 0), else 0
  unsigned mask;
};

__device__ __forceinline__ void dma_patches(__amdgpu_buffer_rsrc_t rs, const PatchAddr& pa, char* raw) {
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    char* dst = raw + r * kRawRow;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)dst, 16, pa.row[r], 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + 1024), 4, pa.row[r] - pa.dl, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + 1280), 4, pa.row[r] + 16, 0, 0, 0);
  }
}

// This lane's raw patch (LDS) → masked → V = Bᵀ d B → V stage row (ch, tile), 6 positions per row
__device__ __forceinline__ void transform_patch(const char* raw, unsigned mask, int lane, float* vd, bool store = true) {
  float d[36];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const char* row = raw + r * kRawRow;
    const float4 m = *reinterpret_cast<const float4*>(row + lane * 16);
    const float l = *reinterpret_cast<const float*>(row + 1024 + lane * 4);
    const float rr = *reinterpret_cast<const float*>(row + 1280 + lane * 4);
    const bool ok = (mask >> r) & 1u;
    d[6 * r + 0] = (ok && (mask & 64u)) ? l : 0.0f;
    d[6 * r + 1] = ok ? m.x : 0.0f;
    d[6 * r + 2] = ok ? m.y : 0.0f;
    d[6 * r + 3] = ok ? m.z : 0.0f;
    d[6 * r + 4] = ok ? m.w : 0.0f;
    d[6 * r + 5] = (ok && (mask & 128u)) ? rr : 0.0f;
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    float t[6];
    bt6(d[c], d[6 + c], d[12 + c], d[18 + c], d[24 + c], d[30 + c], t, 1);
#pragma unroll
    for (int i = 0; i < 6; ++i) d[6 * i + c] = t[i];
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float v[6];
    bt6(d[6 * i], d[6 * i + 1], d[6 * i + 2], d[6 * i + 3], d[6 * i + 4], d[6 * i + 5], v, 1);
    if (store) {
      *reinterpret_cast<float2*>(vd + 6 * i) = make_float2(v[0], v[1]);
      *reinterpret_cast<float2*>(vd + 6 * i + 2) = make_float2(v[2], v[3]);
      *reinterpret_cast<float2*>(vd + 6 * i + 4) = make_float2(v[4], v[5]);
    }
  }
}

// EPI bit 0: + bias[k]; bit 1: + residual (same layout as y).
// MT = output tiles per workgroup: 64 (× 32 output channels), or 32 (× 64 output channels) for
// grids of at most 32 tiles (the UNet's 8² layers at batch 8), where a 64-tile block would run
// half of its MFMAs on empty tiles; lanes 32-63 of the patch waves then only idle.
template <int EPI, int MT>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_f4_kernel(
    const float* __restrict__ x, const float* __restrict__ U, const float* __restrict__ bias,
    const float* __restrict__ res, float* __restrict__ y, int nimg, int C, int K, int H, int W, int tw, int tpi,
    int ntiles, int ntb, int nkb, int kb_major, int csplit, int dbg) {
  // separate LDS objects per buffer, so the compiler can tell a DMA into one buffer from a
  // ds_read of another and does not wait for the DMA before every LDS read
  constexpr int NC = kMT * kNC / MT;                // output channels per workgroup
  constexpr int VS = kCK * MT * kP, US = kCK * NC * kP;
  constexpr int NWM = MT / 16;                      // 16-tile MFMA row blocks
  __shared__ __attribute__((aligned(16))) float V0[VS], V1[VS];   // [kCK][MT][kP]
  __shared__ __attribute__((aligned(16))) float U0[US], U1[US];   // [NC / 32][kCK][32][kP]
  __shared__ __attribute__((aligned(16))) char Raw[4 * kRawWave];   // [4 waves][6 rows][mid | left | right]

  // workgroup → (input-channel split, tile block, channel block); consecutive logical ids share
  // one XCD.  With csplit < C the workgroup sums input channels [sp·csplit, (sp+1)·csplit) only
  // and writes its partial to slab sp of y (the caller's workspace).
  const int G = gridDim.x;
  const int g = blockIdx.x;
  const int Lg = (G % 8 == 0) ? (g % 8) * (G / 8) + g / 8 : g;
  const int sp = Lg / (ntb * nkb);
  const int L = Lg - sp * (ntb * nkb);
  int tb, kb;
  if (kb_major) {
    kb = L / ntb;
    tb = L - kb * ntb;
  } else {
    tb = L / nkb;
    kb = L - tb * nkb;
  }
  const int c0 = sp * csplit;
  y += (size_t)sp * nimg * K * ((EPI & 4) ? (H / 2) * (W / 2) : H * W);   // EPI bit 2: stride-2 output

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv % NWM, wn = wv / NWM;   // this wave's 16 tiles × 16 channels
  const bool patcher = wv < 4;            // waves 0-3: patches of stage channel wv; 4-7: U slices
  const size_t plane = (size_t)H * W;
  PatchAddr pa;
  {
    const int pt = tb * MT + lane;
    const bool pvalid = lane < MT && pt < ntiles;
    int pb = 0, py0 = 0, px0 = 0;
    if (pvalid) {
      pb = pt / tpi;
      const int r = pt - pb * tpi;
      const int ty = r / tw;
      py0 = 4 * ty;
      px0 = 4 * (r - ty * tw);
    }
    const unsigned base = (unsigned)(((size_t)pb * C + (wv & 3)) * plane);
    pa.mask = (px0 > 0 ? 64u : 0u) | (px0 + 4 < W ? 128u : 0u);
    pa.dl = px0 > 0 ? 4u : 0u;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const int yy = py0 - 1 + r;
      if (pvalid && yy >= 0 && yy < H) pa.mask |= 1u << r;
      const int yc = yy < 0 ? 0 : (yy >= H ? H - 1 : yy);
      pa.row[r] = (base + (unsigned)(yc * W + px0)) * 4u;
    }
  }
  // U is stored in 32-channel slices [K / 32][C][32][kP]; a 64-channel block reads two
  const float* Ub = U + ((size_t)(kb * (NC / kNC)) * C + c0) * kNC * kP;
  const size_t uhalf = (size_t)C * kNC * kP;   // floats between consecutive 32-channel slices
  const int nst = csplit / kCK;
  const size_t xfloats = (size_t)nimg * C * plane;
  char* raw = Raw + (wv & 3) * kRawWave;
  const bool vstore = lane < MT;
  const int vrow = ((wv & 3) * MT + (vstore ? lane : 0)) * kP;   // this patcher lane's V row
  // per-stage descriptors: x from the stage's first channel plane, U from the stage's slice
  auto xrsrc = [&](int s) {
    const size_t off = ((size_t)c0 + (size_t)s * kCK) * plane;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(x + off), (short)0, (dbg & 1) ? 0 : (int)((xfloats - off) * 4), 0x00020000);
  };
  auto dma_u = [&](int s, float* ubuf) {
    char* dst = reinterpret_cast<char*>(ubuf);
#pragma unroll
    for (int h = 0; h < NC / kNC; ++h) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(Ub + h * uhalf + (size_t)s * kUs), (short)0, (dbg & 2) ? 0 : kUs * 4, 0x00020000);
#pragma unroll
      for (int c = wv - 4; c < kUChunks; c += 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + h * kUs * 4 + c * 1024), 16, lane * 16, c * 1024,
                                                 0, 0);
    }
  };

  f32x4 acc[kP];
#pragma unroll
  for (int p = 0; p < kP; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: V[0] and U[0] ready, stage 1's raw patches in flight
  if (patcher) {
    dma_patches(xrsrc(0), pa, raw);
    __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) & lgkmcnt(0): this wave's DMA landed
    transform_patch(raw, pa.mask, lane, V0 + vrow, vstore);
    if (nst > 1) dma_patches(xrsrc(1), pa, raw);
  } else {
    dma_u(0, U0);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  // MFMA operands: A = V[k = lane>>4][tile 16·wm + (lane&15)], B = U[k][channel 16·wn + (lane&15)]
  const int aoff = ((lane >> 4) * MT + wm * 16 + (lane & 15)) * kP;
  const int boff = (wn >> 1) * kUs + ((lane >> 4) * kNC + (wn & 1) * 16 + (lane & 15)) * kP;
  // one stage: prepare stage s+1 into (vn, un), MFMAs on (vc, uc); the loop is unrolled by two
  // so every buffer is a fixed LDS object in each half
  auto phase = [&](int s, const float* vc, const float* uc, float* vn, float* un) {
    if (s + 1 < nst) {
      if (patcher) {
        if (!(dbg & 4)) transform_patch(raw, pa.mask, lane, vn + vrow, vstore);
        if (s + 2 < nst) dma_patches(xrsrc(s + 2), pa, raw);
      } else {
        dma_u(s + 1, un);
      }
    }
    const float* va = vc + aoff;
    const float* ub = uc + boff;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      if (dbg & 8) break;
      const float4 a = *reinterpret_cast<const float4*>(va + 4 * q);
      const float4 b = *reinterpret_cast<const float4*>(ub + 4 * q);
      acc[4 * q + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc[4 * q + 0], 0, 0, 0);
      acc[4 * q + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc[4 * q + 1], 0, 0, 0);
      acc[4 * q + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc[4 * q + 2], 0, 0, 0);
      acc[4 * q + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc[4 * q + 3], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);   // this wave's DMA for the next stage has landed
    __syncthreads();
  };
  for (int s = 0; s < nst; s += 2) {
    phase(s, V0, U0, V1, U1);
    if (s + 1 < nst) phase(s + 1, V1, U1, V0, U0);
  }

  // epilogue: lane holds rows 4·(lane>>4)+r (tiles) × column lane&15 (channel) of every position
  const int k = kb * NC + wn * 16 + (lane & 15);
  const float bv = (EPI & 1) ? bias[k] : 0.0f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int t = tb * MT + wm * 16 + 4 * (lane >> 4) + r;
    if (t >= ntiles) continue;
    float m[36], o[16];
#pragma unroll
    for (int p = 0; p < kP; ++p) m[p] = acc[p][r];
    output_transform(m, o);
    const int b = t / tpi;
    const int rr = t - b * tpi;
    const int ty = rr / tw;
    const int tx = rr - ty * tw;
    const size_t off = ((size_t)b * K + k) * plane + (size_t)(4 * ty) * W + 4 * tx;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 val = make_float4(o[4 * i] + bv, o[4 * i + 1] + bv, o[4 * i + 2] + bv, o[4 * i + 3] + bv);
      if (EPI & 2) {
        const float4 rv = *reinterpret_cast<const float4*>(res + off + (size_t)i * W);
        val.x += rv.x;
        val.y += rv.y;
        val.z += rv.z;
        val.w += rv.w;
      }
      *reinterpret_cast<float4*>(y + off + (size_t)i * W) = val;
    }
  }
}

// U[kb][c][k%32][36] = G g Gᵀ in fp64, g = w[k][c] (flip 0) or rot180(w[c][k]) (flip 1)
__global__ void wino_weights_kernel(const float* __restrict__ w, int K, int C, int flip, float* __restrict__ U) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)K * C) return;
  const int k = (int)(i / C), c = (int)(i - (long long)k * C);
  double g[9];
  for (int u = 0; u < 3; ++u)
    for (int v = 0; v < 3; ++v)
      g[3 * u + v] = flip ? (double)w[((size_t)c * K + k) * 9 + (2 - u) * 3 + (2 - v)]
                          : (double)w[((size_t)k * C + c) * 9 + u * 3 + v];
  const double Gm[6][3] = {{1.0, 0.0, 0.0},
                           {1.0 / 3, 1.0 / 3, 1.0 / 3},
                           {-1.0 / 3, 1.0 / 3, -1.0 / 3},
                           {-16.0 / 15, -8.0 / 15, -4.0 / 15},
                           {1.0 / 15, -2.0 / 15, 4.0 / 15},
                           {0.0, 0.0, 1.0}};
  double t[6][3];
  for (int a = 0; a < 6; ++a)
    for (int v = 0; v < 3; ++v) t[a][v] = Gm[a][0] * g[v] + Gm[a][1] * g[3 + v] + Gm[a][2] * g[6 + v];
  float* out = U + (((size_t)(k / kNC) * C + c) * kNC + (k % kNC)) * kP;
  for (int a = 0; a < 6; ++a)
    for (int b = 0; b < 6; ++b) out[6 * a + b] = (float)(t[a][0] * Gm[b][0] + t[a][1] * Gm[b][1] + t[a][2] * Gm[b][2]);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int skp_wino_weights(const float* w, int K, int C, int flip, float* U, void* stream) {
  SKP_CHECK_ARG(w && U, "null pointer");
  SKP_CHECK_ARG(K > 0 && C > 0, "non-positive shape");
  SKP_CHECK_ARG(K % kNC == 0, "output channels must be a multiple of 32");
  const long long n = (long long)K * C;
  hipLaunchKernelGGL(wino_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), w, K, C,
                     flip, U);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

namespace {

// y = Σ_s ws[s] + bias[k] + residual over (B, K, HW), float4 lanes (HW % 4 == 0)
__global__ void splitk_reduce_kernel(const float4* __restrict__ ws, int nsplit, long long n4, int K, int hw4,
                                     const float* __restrict__ bias, const float4* __restrict__ res,
                                     float4* __restrict__ y) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 v = ws[i];
  for (int s = 1; s < nsplit; ++s) {
    const float4 p = ws[(long long)s * n4 + i];
    v.x += p.x;
    v.y += p.y;
    v.z += p.z;
    v.w += p.w;
  }
  if (bias) {
    const float b = bias[(i / hw4) % K];
    v.x += b;
    v.y += b;
    v.z += b;
    v.w += b;
  }
  if (res) {
    const float4 r = res[i];
    v.x += r.x;
    v.y += r.y;
    v.z += r.z;
    v.w += r.w;
  }
  y[i] = v;
}

int splitk_reduce(const float* ws, int nsplit, int B, int K, int HW, const float* bias, const float* residual,
                  float* y, hipStream_t st) {
  const long long n4 = (long long)B * K * HW / 4;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(ws), nsplit, n4, K, HW / 4, bias,
                     reinterpret_cast<const float4*>(residual), reinterpret_cast<float4*>(y));
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

}  // namespace

extern "C" int skp_conv3x3_wino(const float* x, const float* U, const float* bias, const float* residual, float* y,
                                int B, int C, int K, int H, int W, int nsplit, float* ws, void* stream) {
  SKP_CHECK_ARG(x && U && y, "null pointer");
  SKP_CHECK_ARG(B > 0 && C > 0 && K > 0 && H > 0 && W > 0, "non-positive shape");
  SKP_CHECK_ARG(C % kCK == 0, "input channels must be a multiple of 4");
  SKP_CHECK_ARG(K % kNC == 0, "output channels must be a multiple of 32");
  SKP_CHECK_ARG(H % 4 == 0 && W % 4 == 0, "H and W must be multiples of 4");
  SKP_CHECK_ARG(nsplit >= 1 && C % (kCK * nsplit) == 0, "nsplit must divide C into multiples of 4");
  SKP_CHECK_ARG(nsplit == 1 || ws, "split-K needs a workspace of nsplit·B·K·H·W floats");
  SKP_CHECK_ARG(aligned16(x) && aligned16(U) && aligned16(y) && (!residual || aligned16(residual)) &&
                    (!ws || aligned16(ws)),
                "tensors must be 16-byte aligned");
  const int tw = W / 4, tpi = (H / 4) * tw;
  const long long ntiles = (long long)B * tpi;
  SKP_CHECK_ARG(ntiles <= 0x7fffffffLL - kMT, "too many tiles");
  SKP_CHECK_ARG((long long)B * C * H * W * 4 < 0x7fffffffLL, "input larger than 2 GiB (32-bit buffer offsets)");
  // at most 32 tiles (8² at batch 8): 32-tile × 64-channel workgroups (ops.wino_conv's planner
  // mirrors this rule)
  const bool wide = ntiles <= 32 && K % 64 == 0;
  const int mt = wide ? 32 : kMT;
  const int ntb = (int)((ntiles + mt - 1) / mt), nkb = K / (wide ? 64 : kNC);
  SKP_CHECK_ARG((long long)ntb * nkb * nsplit <= 0x7fffffffLL, "grid too large");
  // one channel block's U slice is C·32·36·4 B; keep all of U on an L2 slice when it fits
  const long long ubytes = (long long)K * C * kP * 4;
  const int kb_major = ubytes > (2LL << 20);
  const int epi = nsplit > 1 ? 0 : (bias ? 1 : 0) | (residual ? 2 : 0);
  float* out = nsplit > 1 ? ws : y;
  const int dbg = SKP_WINO_DEBUG;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(ntb * nkb * nsplit));
#define SKP_WG(E)                                                                                                    \
  if (wide)                                                                                                          \
    hipLaunchKernelGGL((wino_f4_kernel<E, 32>), grid, dim3(kThreads), 0, st, x, U, bias, residual, out, B, C, K, H, W, \
                       tw, tpi, (int)ntiles, ntb, nkb, kb_major, C / nsplit, dbg);                                    \
  else                                                                                                               \
    hipLaunchKernelGGL((wino_f4_kernel<E, 64>), grid, dim3(kThreads), 0, st, x, U, bias, residual, out, B, C, K, H, W, \
                       tw, tpi, (int)ntiles, ntb, nkb, kb_major, C / nsplit, dbg)
  switch (epi) {
    case 0: SKP_WG(0); break;
    case 1: SKP_WG(1); break;
    case 2: SKP_WG(2); break;
    default: SKP_WG(3); break;
  }
#undef SKP_WG
  SKP_LAUNCH_CHECK();
  if (nsplit > 1) return splitk_reduce(ws, nsplit, B, K, H * W, bias, residual, y, st);
  return SKP_OK;
}

// ================================================================================================
// Winograd F(4×4, 3×3), region-staged version for H and W multiples of 32 (every VAE-encoder
// layer at 512² input and the UNet's 64² / 32² layers).
//
// The kernel above is bound by its one-deep pipeline: every stage waits for LDS-DMA it issued
// in the same stage (≈1 µs under load, about one stage of MFMA work), and with neither
// transforms nor MFMAs it still takes half its time.  This one keeps three stages in flight:
//   - a workgroup owns an 8×8 block of output tiles (32×32 pixels) × 32 output channels; per
//     stage of 4 input channels it DMAs the block's 34×34-pixel input region as rows of ten
//     16-byte chunks (columns x0-4 … x0+35; rows and chunks outside the image load as zeros —
//     out-of-range buffer offsets — so the zero padding costs no masking) and the stage's U
//     slice, into 3-slot LDS rings, two stages ahead of use;
//   - the transformed input never goes through LDS: lane (tile, channel) of a wave reads its
//     own 6×6 patch (three ds_read_b128 per row) and computes the V values that are exactly its
//     MFMA A operand.  The two waves of a SIMD (w, w+4) share the 16 tiles and split the 36
//     positions by transform rows (0-2 / 3-5), so no transform work is repeated: each runs half
//     of the column pass and half of the row pass;
//   - a wave owns 16 tiles × 32 channels × 18 positions (2 MFMA blocks, 144 accumulators) and
//     transforms stage s+1 while its MFMAs run on stage s (the A operands are double-buffered
//     in registers);
//   - one barrier per stage; the epilogue applies the output transform to each half's rows and
//     the partner waves exchange the half-sums through LDS (two rounds of 8 KB per wave).
// ================================================================================================
namespace {
namespace w2 {

constexpr int kNC = 32;                    // output channels per workgroup
constexpr int kCK = 4;                     // input channels per stage
// Block geometry: a workgroup's 64 output tiles are TXB×TXB tiles of each of NI images' regions.
//   TXB 8: a 32×32-pixel block of one image (H, W multiples of 32); region 34 rows × 10 chunks
//   TXB 4: four whole 16×16 images; region 18 rows × 6 chunks per image
// The channel stride (floats) makes the patch reads' ds_read_b128 lane groups conflict-free.
template <int TXB>
struct Geo;
template <>
struct Geo<8> {
  static constexpr int NI = 1, RR = 34, RC = 10, CHF = 1408;
};
template <>
struct Geo<4> {
  static constexpr int NI = 4, RR = 18, RC = 6, CHF = 1744;
};
// NW = 4 with TXB 8: a half-height block (8 × 4 tiles = 32 × 16 pixels, 4 waves), so that two
// workgroups share a CU and one's prologue / epilogue overlaps the other's stage loop
template <int TXB, int NW>
struct GeoN : Geo<TXB> {};
template <>
struct GeoN<8, 4> {
  static constexpr int NI = 1, RR = 18, RC = 10, CHF = 768;   // same bank residues as 1408
};
// NW = 4 with TXB 4: two whole 16×16 images per workgroup (4 waves); CHF/4 ≡ 12 (mod 16) keeps
// the patch reads' ds_read_b128 lane groups conflict-free like 1744 (≡ 4)
template <>
struct GeoN<4, 4> {
  static constexpr int NI = 2, RR = 18, RC = 6, CHF = 880;
};
template <int TXB, int NW = 8>
struct GeoT : GeoN<TXB, NW> {
  using GeoN<TXB, NW>::NI;
  using GeoN<TXB, NW>::RR;
  using GeoN<TXB, NW>::RC;
  using GeoN<TXB, NW>::CHF;
  static constexpr int RF = 4 * RC;                                   // floats per region row
  static constexpr int RAWF = (4 * CHF + 255) / 256 * 256;            // raw slot, whole 1-KB chunks
  static constexpr int RAW_INSTR = RAWF / 256;
  static_assert(NI * RR * RF <= CHF, "channel region");
};
constexpr int kUP = 40;                    // floats per (input, output channel) U row
constexpr int kUF = kCK * kNC * kUP;       // 5120 floats = 20 KB per U slot
constexpr int kUInstr = kUF / 256;         // 20
constexpr unsigned kOOB = 0x80000000u;     // buffer offset past any num_records (< 2 GiB): loads 0
static_assert(kUF % 256 == 0, "whole 1-KB chunks");
static_assert((4 * GeoT<8>::RAWF + 3 * kUF) * 4 <= 160 * 1024 && 3 * (GeoT<4>::RAWF + kUF) * 4 <= 160 * 1024, "LDS");
static_assert(2 * 8 * 1024 <= kUF * 4, "epilogue exchange: two waves' 8 KB per ring buffer");

// Bᵀ (rows i = transform row, columns a = patch row) for the points (0, 1, -1, 1/2, -2, ∞)
__device__ constexpr float kBt[6][6] = {{1.f, -1.5f, -2.f, 1.5f, 1.f, 0.f},  {0.f, -1.f, 0.5f, 2.5f, 1.f, 0.f},
                                        {0.f, 1.f, -2.5f, 0.5f, 1.f, 0.f},  {0.f, -2.f, -1.f, 2.f, 1.f, 0.f},
                                        {0.f, 0.5f, -1.f, -0.5f, 1.f, 0.f}, {0.f, 1.f, -1.5f, -2.f, 1.5f, 1.f}};
// Aᵀ (4 outputs × 6 positions)
__device__ constexpr float kAt[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                                        {0.f, 1.f, -1.f, 0.5f, -2.f, 0.f},
                                        {0.f, 1.f, 1.f, 0.25f, 4.f, 0.f},
                                        {0.f, 1.f, -1.f, 0.125f, -8.f, 1.f}};

#ifndef SKP_W2_PACKED
#define SKP_W2_PACKED 1   // 0: the scalar half_transform (A/B build)
#endif
#if SKP_W2_PACKED
#define W2_TRANSFORM half_transform_pk
#else
#define W2_TRANSFORM half_transform
#endif

// s_waitcnt vmcnt(n) with expcnt / lgkmcnt left alone (gfx9 encoding)
#define W2_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | (7 << 4) | (15 << 8))

// Transform rows 3H..3H+2 of V = Bᵀ d B for this lane's patch (region rows at `raw`, the
// patch's first row; columns: .w of chunk 0, chunk 1, .x of chunk 2) → a[18] = V[3H+ii][j].
template <int H, int RF>
__device__ __forceinline__ void half_transform(const float* raw, float* a) {
  float t[3][6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const float4 c0 = *reinterpret_cast<const float4*>(raw + r * RF);
    const float4 c1 = *reinterpret_cast<const float4*>(raw + r * RF + 4);
    const float4 c2 = *reinterpret_cast<const float4*>(raw + r * RF + 8);
    const float d[6] = {c0.w, c1.x, c1.y, c1.z, c1.w, c2.x};
#pragma unroll
    for (int ii = 0; ii < 3; ++ii) {
      const float c = kBt[3 * H + ii][r];
      if (c == 0.0f) continue;
      bool first = true;   // the first nonzero coefficient of row 3H+ii (compile time)
#pragma unroll
      for (int rp = 0; rp < r; ++rp)
        if (kBt[3 * H + ii][rp] != 0.0f) first = false;
#pragma unroll
      for (int b = 0; b < 6; ++b)
        t[ii][b] = first ? ((c == 1.0f) ? d[b] : c * d[b]) : ((c == 1.0f) ? t[ii][b] + d[b] : fmaf(c, d[b], t[ii][b]));
    }
    // keep chunks 0 and 2 whole: with one component used the compiler narrows them to
    // ds_read_b32, 4-way bank-conflicted at this layout (ds_read_b128 is conflict-free)
    asm volatile("" ::"v"(c0.x), "v"(c0.y), "v"(c0.z), "v"(c2.y), "v"(c2.z), "v"(c2.w));
  }
#pragma unroll
  for (int ii = 0; ii < 3; ++ii) bt6(t[ii][0], t[ii][1], t[ii][2], t[ii][3], t[ii][4], t[ii][5], a + 6 * ii, 1);
}

typedef float f2 __attribute__((ext_vector_type(2)));

// y = Bᵀ x with shared differences: 16 operations instead of 20 (e, f, g, h reused)
template <typename T>
__device__ __forceinline__ void bt6_shared(T a0, T a1, T a2, T a3, T a4, T a5, T* y) {
  const T e = a4 - a2, f = a3 - a1, g = a2 + a3, h = a3 - a2;
  y[0] = __builtin_elementwise_fma((T)1.5f, f, (a0 + e) - a2);
  y[1] = __builtin_elementwise_fma((T)1.5f, g, e + f);
  y[2] = __builtin_elementwise_fma((T)1.5f, h, e - f);
  y[3] = __builtin_elementwise_fma((T)2.0f, f, e);
  y[4] = __builtin_elementwise_fma((T)-0.5f, f, e);
  y[5] = __builtin_elementwise_fma((T)1.5f, e, __builtin_elementwise_fma((T)-2.0f, f, a5 - a1));
}

// Packed form of half_transform (v_pk_* f32): the column pass runs on column pairs
// (1,2), (3,4), (0,5) — the first two are halves of the middle 16-B chunk, the third one
// v_pk_mov per row — streaming the patch rows through shared differences (9 / 7 operations
// per pair for rows 0-2 / 3-5 instead of 10); the row pass packs transform rows 3H and 3H+1
// (pairs re-formed per column) and runs row 3H+2 unpacked, both with the shared-difference
// Bᵀ.  ≈80 VALU instructions per patch half and stage instead of ≈109.
template <int H, int RF>
__device__ __forceinline__ void half_transform_pk(const float* raw, float* a) {
  f2 t[3][3];   // t[ii][p]: column pair p of transform row 3H+ii
  f2 k0[3], k1[3], k2[3], k3[3];   // streamed partial terms (per column pair)
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    if (H == 1 && r == 0) continue;   // Bᵀ rows 3-5 do not read patch row 0
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(raw + r * RF);
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(raw + r * RF + 4);
    const f32x4 c2 = *reinterpret_cast<const f32x4*>(raw + r * RF + 8);
    const f2 d[3] = {__builtin_shufflevector(c1, c1, 0, 1), __builtin_shufflevector(c1, c1, 2, 3),
                     __builtin_shufflevector(c0, c2, 3, 4)};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      if (H == 0) {
        // s = −a2 + 1.5a3 + a4, q = −a1 + 1.5a2 + a3: rows 1, 2 = s ± q, row 0 = a0 − 1.5a1 + (s − a2)
        if (r == 0) k0[p] = d[p];
        if (r == 1) { k1[p] = d[p]; k0[p] = __builtin_elementwise_fma((f2)-1.5f, d[p], k0[p]); }
        if (r == 2) { k2[p] = d[p]; k3[p] = __builtin_elementwise_fma((f2)1.5f, d[p], -k1[p]); }
        if (r == 3) { k1[p] = __builtin_elementwise_fma((f2)1.5f, d[p], -k2[p]); k3[p] = k3[p] + d[p]; }
        if (r == 4) {
          const f2 sv = k1[p] + d[p];
          t[0][p] = k0[p] + (sv - k2[p]);
          t[1][p] = sv + k3[p];
          t[2][p] = sv - k3[p];
        }
      } else {
        // e = a4 − a2, f = a3 − a1: row 3 = e + 2f, row 4 = e − f/2, row 5 = 1.5e − 2f − a1 + a5
        if (r == 1) k0[p] = d[p];
        if (r == 2) k1[p] = d[p];
        if (r == 3) { k2[p] = d[p] - k0[p]; k3[p] = __builtin_elementwise_fma((f2)-2.0f, k2[p], -k0[p]); }
        if (r == 4) {
          const f2 e = d[p] - k1[p];
          t[0][p] = __builtin_elementwise_fma((f2)2.0f, k2[p], e);
          t[1][p] = __builtin_elementwise_fma((f2)-0.5f, k2[p], e);
          k3[p] = __builtin_elementwise_fma((f2)1.5f, e, k3[p]);
        }
        if (r == 5) t[2][p] = k3[p] + d[p];
      }
    }
    asm volatile("" ::"v"(c0.x), "v"(c0.y), "v"(c0.z), "v"(c2.y), "v"(c2.z), "v"(c2.w));
  }
  // row pass: column b of row ii is t[ii][0] = (b1, b2), t[ii][1] = (b3, b4), t[ii][2] = (b0, b5)
  const f2 u0 = __builtin_shufflevector(t[0][2], t[1][2], 0, 2), u1 = __builtin_shufflevector(t[0][0], t[1][0], 0, 2);
  const f2 u2 = __builtin_shufflevector(t[0][0], t[1][0], 1, 3), u3 = __builtin_shufflevector(t[0][1], t[1][1], 0, 2);
  const f2 u4 = __builtin_shufflevector(t[0][1], t[1][1], 1, 3), u5 = __builtin_shufflevector(t[0][2], t[1][2], 1, 3);
  f2 y01[6];
  bt6_shared<f2>(u0, u1, u2, u3, u4, u5, y01);
  float y2[6];
  bt6_shared<float>(t[2][2].x, t[2][0].x, t[2][0].y, t[2][1].x, t[2][1].y, t[2][2].y, y2);
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    a[j] = y01[j].x;
    a[6 + j] = y01[j].y;
    a[12 + j] = y2[j];
  }
}

// partial output tile of rows 3H..3H+2 of M (m[18] = M[3H+ii][j]) → y[16] (row-major 4×4)
template <int H>
__device__ __forceinline__ void half_output(const float* m, float* y) {
  float s[3][4];
#pragma unroll
  for (int ii = 0; ii < 3; ++ii) at6(m[6 * ii], m[6 * ii + 1], m[6 * ii + 2], m[6 * ii + 3], m[6 * ii + 4], m[6 * ii + 5], s[ii], 1);
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float v = 0.0f;
      bool first = true;
#pragma unroll
      for (int ii = 0; ii < 3; ++ii) {
        const float a = kAt[r][3 * H + ii];
        if (a == 0.0f) continue;
        v = first ? ((a == 1.0f) ? s[ii][c] : a * s[ii][c]) : fmaf(a, s[ii][c], v);
        first = false;
      }
      y[4 * r + c] = v;
    }
}

}  // namespace w2

struct W2Smem {
  float *R0, *R1, *R2, *R3, *U0, *U1, *U2;
};

// s_waitcnt vmcnt(n) for a wave-uniform n (the per-wave DMA instruction counts differ)
__device__ __forceinline__ void w2_vmcnt(int n) {
  switch (n) {
    case 0: W2_VMCNT(0); break;
    case 1: W2_VMCNT(1); break;
    case 2: W2_VMCNT(2); break;
    case 3: W2_VMCNT(3); break;
    case 4: W2_VMCNT(4); break;
    case 5: W2_VMCNT(5); break;
    case 6: W2_VMCNT(6); break;
    case 7: W2_VMCNT(7); break;
    case 8: W2_VMCNT(8); break;
    case 9: W2_VMCNT(9); break;
    case 10: W2_VMCNT(10); break;
    case 11: W2_VMCNT(11); break;
    case 12: W2_VMCNT(12); break;
    case 13: W2_VMCNT(13); break;
    case 14: W2_VMCNT(14); break;
    case 15: W2_VMCNT(15); break;
    default: W2_VMCNT(0); break;
  }
}

#ifndef SKP_W2_RS4
#define SKP_W2_RS4 0   // 1: four raw-input slots for the 32×32 geometry (lead 3; measured 1-2% slower)
#endif

// One wave's whole program for transform half HH (rows 3HH..3HH+2); the kernel branches once
// on the wave's half so the stage loop is straight-line code for each.
template <int EPI, int HH, int TXB, int NW>
__device__ __forceinline__ void wino2_body(const W2Smem& sm, const float* __restrict__ x, const float* __restrict__ U,
                                           const float* __restrict__ bias, const float* __restrict__ res,
                                           float* __restrict__ y, int C, int K, int H, int W, int img, int x0,
                                           int y0, int kb, int c0, int csplit, int wv, int dbg,
                                           float2* __restrict__ gnp) {
  using Geo = w2::GeoT<TXB, NW>;
  constexpr int kChF = Geo::CHF, kRowF = Geo::RF, kRawInstr = Geo::RAW_INSTR, NI = Geo::NI, RR = Geo::RR,
                RC = Geo::RC;
  constexpr int kInstr = kRawInstr + w2::kUInstr;
  constexpr int kMaxRaw = (kRawInstr + NW - 1) / NW;
  constexpr int kMaxU = (w2::kUInstr + NW - 1) / NW + 1;
  constexpr int NT = NW * WAVE;
  // weight ring: 3 slots (lead 2) with 8 waves; 2 (lead 1) in the half-height form, whose LDS must
  // leave room for a second workgroup on the CU
  constexpr int US = NW == 4 ? 2 : 3;
  using w2::kUF;
  using w2::kUP;
  // raw-input ring of RS slots (lead RS − 1 stages: the input streams from HBM), weight ring
  // of 3 (lead 2: the weights are re-read by every tile block and hit L2)
  constexpr int RS = (TXB == 4 && NW == 4) ? 2 : (TXB == 8 && NW == 8 && SKP_W2_RS4) ? 4 : 3;
  float *R0 = sm.R0, *R1 = sm.R1, *R2 = sm.R2, *U0 = sm.U0, *U1 = sm.U1, *U2 = sm.U2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wm = wv % (NW / 2);
  const size_t plane = (size_t)H * W;
  const size_t ximg = (size_t)img * C * plane;

  // this wave's DMA chunks of a stage: chunk g = wv + 8m (the raw slot's chunks, then U's 20);
  // raw chunk → (channel, image of the block, region row, 16-B column chunk)
  unsigned voff[kMaxRaw];
  int nraw = 0;
#pragma unroll
  for (int m = 0; m < kMaxRaw; ++m) {
    const int gi = wv + NW * m;
    voff[m] = w2::kOOB;
    if (gi < kRawInstr) {
      ++nraw;
      const int f = 64 * gi + lane;   // 16-B chunk of the slot
      const int ch = f / (kChF / 4);
      const int e = f - ch * (kChF / 4);
      const int ii = e / (RR * RC), rem = e - ii * (RR * RC);
      const int row = rem / RC, c4 = rem - row * RC;
      const int yy = y0 - 1 + row, xx = x0 - 4 + 4 * c4;
      if (ch < w2::kCK && ii < NI && yy >= 0 && yy < H && xx >= 0 && xx < W)
        voff[m] = (unsigned)((ximg + ((size_t)ii * C + ch) * plane + (size_t)yy * W + xx) * 4);
    }
  }
  const int nuw = (kInstr - 1 - wv) / NW + 1 - nraw;  // U chunks of this wave
  const int ufirst = wv + NW * nraw - kRawInstr;      // its first U chunk
  // vmcnt allowances (in-order counter; per step the wave issues U(s+2) then raw(s+RS)):
  // top of step s needs U(s) and raw(s+1) landed; the prologue needs raw(0)
  // (US = 2: per step U(s+1) then raw(s+3); the top of step s needs U(s) and raw(s+1), the prologue raw(0))
  // (RS = 2, US = 2: per step U(s+1) then raw(s+2), the top of step s waits for both of the
  // previous step's; the prologue issues raw(0), U(0), raw(1) and waits for raw(0))
  const int allow_step = RS == 2 ? 0 : US == 2 ? nraw : RS == 4 ? nuw + 2 * nraw : nuw + nraw;
  const int allow_pro = RS == 2 ? nuw + nraw : US == 2 ? nuw + 2 * nraw : RS == 4 ? 2 * nuw + 3 * nraw : 2 * nuw + 2 * nraw;
  const size_t xend = (size_t)(img + NI) * C * plane; // the buffer ends with the block's last image
  const float* Ub = U + ((size_t)kb * C + c0) * w2::kNC * kUP;
  const int nst = csplit / w2::kCK;

  // raw(t) → raw slot t % RS, U(t) → U slot t % 3
  auto issue_raw = [&](int t, float* rs_lds) {
    const bool ok = t < nst;
    const size_t off = ((size_t)c0 + (size_t)(ok ? t : 0) * w2::kCK) * plane;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + off), (short)0, ok ? (int)((xend - off) * 4) : 0, 0x00020000);
#pragma unroll
    for (int m = 0; m < kMaxRaw; ++m)
      if (m < nraw && !(dbg & 4))
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(rs_lds + 256 * (wv + NW * m)), 16, voff[m], 0, 0, 0);
  };
  auto issue_u = [&](int t, float* us_lds) {
    const __amdgpu_buffer_rsrc_t ru =
        __builtin_amdgcn_make_buffer_rsrc((void*)(Ub + (size_t)t * kUF), (short)0, kUF * 4, 0x00020000);
#pragma unroll
    for (int m = 0; m < kMaxU; ++m)
      if (m < nuw && !(dbg & 8)) {
        const int q = ufirst + NW * m;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ru, (lds_ptr_t)(us_lds + 256 * q), 16, lane * 16, q * 1024, 0, 0);
      }
  };

  // lane → (tile, stage channel) = its A-operand row; the patch's first row in the region.
  // TXB 8: wave wm has tile rows 2wm, 2wm+1; TXB 4: wave wm has image wm of the block.
  const int kc = lane >> 4;
  const int tx = lane & (TXB - 1);
  const int ty = TXB == 8 ? 2 * wm + ((lane >> 3) & 1) : (lane >> 2) & 3;
  const int roff = kc * kChF + (TXB == 8 ? 0 : wm * RR * kRowF) + 4 * ty * kRowF + 4 * tx;
  // B operand: U[kc][16 blk + (lane & 15)][18 HH + q] (rows padded to 40, halves at 0 and 20)
  const int uoff = (kc * w2::kNC + (lane & 15)) * kUP + 20 * HH;

  f32x4 acc[2][18];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int q = 0; q < 18; ++q) acc[b][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a0[18], a1[18];   // A operands of the even / odd stages (no copies between stages)

  auto mfmas = [&](const float* us, const float (&acur)[18]) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const float* ub = us + uoff + b * 16 * kUP;
      float u[18];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(ub + 4 * j);
        u[4 * j] = v.x;
        u[4 * j + 1] = v.y;
        u[4 * j + 2] = v.z;
        u[4 * j + 3] = v.w;
      }
      const float2 v2 = *reinterpret_cast<const float2*>(ub + 16);
      u[16] = v2.x;
      u[17] = v2.y;
#pragma unroll
      for (int q = 0; q < 18; ++q) acc[b][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(acur[q], u[q], acc[b][q], 0, 0, 0);
    }
  };

  // prologue: the DMAs of "steps" −RS..−1 (raw(0..RS−1), U(0), U(1)) in step order; wait for
  // raw(0) and transform it
  issue_raw(0, R0);
  if (RS == 4) issue_raw(1, R1);
  issue_u(0, U0);
  if (RS >= 3) issue_raw(RS - 2, RS == 4 ? R2 : R1);
  if (US == 3 && nst > 1) issue_u(1, U1);
  issue_raw(RS - 1, RS == 4 ? sm.R3 : RS == 3 ? R2 : R1);
  w2_vmcnt(nst > 1 ? allow_pro : 0);
  __syncthreads();
  w2::W2_TRANSFORM<HH, kRowF>(R0 + roff, a0);

  // stage s: wait for U(s) and raw(s+1); barrier; issue U(s+2) and raw(s+RS) into the slots
  // freed by stage s-1; transform raw(s+1) (slot (s+1)%RS) and run the MFMAs on U(s) (slot
  // s%3).  The SIMD partners (waves w, w+4: the two halves) do these in opposite orders.
  auto step = [&](int s, float* Rn, float* Us, float* Ri, float* Ui, const float (&acur)[18], float (&anext)[18]) {
    w2_vmcnt(s + 1 < nst ? allow_step : 0);
    __syncthreads();
    if (s + US - 1 < nst) issue_u(s + US - 1, Ui);
    issue_raw(s + RS, Ri);   // past the last stage: empty (zero-length) loads keep the counts
    const bool tr = s + 1 < nst && !(dbg & 1);
    if (HH == 0) {
      if (tr) w2::W2_TRANSFORM<HH, kRowF>(Rn + roff, anext);
      if (!(dbg & 2)) mfmas(Us, acur);
    } else {
      if (!(dbg & 2)) mfmas(Us, acur);
      if (tr) w2::W2_TRANSFORM<HH, kRowF>(Rn + roff, anext);
    }
  };
  // unrolled by lcm(RS, 3, 2): raw slot s%RS, U slot s%3, A-operand buffer s%2
  constexpr int PER = RS == 4 ? 12 : RS == 2 ? 2 : 6;
  float* const Rsl[4] = {R0, R1, R2, sm.R3};
  float* const Usl[3] = {U0, U1, U2};
  for (int s0 = 0; s0 < ((dbg & 16) ? 0 : nst); s0 += PER) {
    step(s0, Rsl[1 % RS], Usl[0], Rsl[0], Usl[US - 1], a0, a1);
#pragma unroll
    for (int j = 1; j < PER; ++j) {
      if (s0 + j < nst) {
        if ((j & 1) == 0) step(s0 + j, Rsl[(j + 1) % RS], Usl[j % US], Rsl[j % RS], Usl[(j + US - 1) % US], a0, a1);
        else step(s0 + j, Rsl[(j + 1) % RS], Usl[j % US], Rsl[j % RS], Usl[(j + US - 1) % US], a1, a0);
      }
    }
  }

  // epilogue: lane holds tiles 4(lane>>4)+r of the wave's 16 (ty = 2wm + (lane>>5),
  // tx = 4((lane>>4)&1) + r) × channel 16 blk + (lane&15), rows 3HH..3HH+2 of M.  Per block of 16
  // channels: the other half's waves stage their partial tiles in LDS ([ch][32 rows][32 px]),
  // this half's waves add theirs in place, then every thread stores whole 128-B rows.
  W2_VMCNT(0);
  __syncthreads();
  if (dbg & 32) return;
  // channel c of a block: a 32×32-float plane in R0/R1/R2/U0 (four channels each, skewed by 16
  // floats per buffer so the 8-lane store groups hit distinct banks)
  constexpr int PH = (TXB == 8 && NW == 4) ? 16 : 32;   // plane rows (TXB 8: the block's pixel rows)
  // plane stride: TXB 8 the block's PH × 32 pixels, TXB 4 its NI 16×16 images (+4 skew); with a
  // 2-slot raw ring the third plane buffer is U1 (no R2)
  constexpr int PLS = (TXB == 8 ? PH * 32 : NI * 256) + 4;
  float* const P2 = RS == 2 ? U1 : R2;
  auto plane_of = [&](int c) -> float* {
    float* b = (c >> 2) == 0 ? R0 : (c >> 2) == 1 ? R1 : (c >> 2) == 2 ? P2 : U0;
    return b + (c & 3) * PLS + (c >> 2) * 16;
  };
  // this lane's output tile row within the 1024-float plane: TXB 8: tiles (2wm + lane>>5, 4((lane>>4)&1)
  // + r) of the 32×32 block; TXB 4: image wm (256 floats), tile row lane>>4, tiles r = 0..3
  float* pl = plane_of(lane & 15);
  const int pbase = TXB == 8 ? (4 * (2 * wm + (lane >> 5))) * 32 + 4 * (4 * ((lane >> 4) & 1))
                             : wm * 256 + (4 * (lane >> 4)) * 16;
  constexpr int PW = TXB == 8 ? 32 : 16;   // plane row width
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    if (HH != blk) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float m[18], o[16];
#pragma unroll
        for (int q = 0; q < 18; ++q) m[q] = acc[blk][q][r];
        w2::half_output<HH>(m, o);
#pragma unroll
        for (int f = 0; f < 4; ++f)
          *reinterpret_cast<float4*>(pl + pbase + f * PW + 4 * r) =
              make_float4(o[4 * f], o[4 * f + 1], o[4 * f + 2], o[4 * f + 3]);
      }
    }
    __syncthreads();
    if (HH == blk) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float m[18], o[16];
#pragma unroll
        for (int q = 0; q < 18; ++q) m[q] = acc[blk][q][r];
        w2::half_output<HH>(m, o);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          float4* d = reinterpret_cast<float4*>(pl + pbase + f * PW + 4 * r);
          const float4 p = *d;
          *d = make_float4(o[4 * f] + p.x, o[4 * f + 1] + p.y, o[4 * f + 2] + p.z, o[4 * f + 3] + p.w);
        }
      }
    }
    __syncthreads();
    if constexpr ((EPI & 4) != 0) {
      // stride-2 output (EPI bit 2, TXB 8): the block's odd rows / columns, a 16×16 block of the
      // (H/2, W/2) output per channel = 16 channels × 64 float4, two per thread
      static_assert(TXB == 8 && (EPI & 2) == 0, "stride-2 output: 32-wide blocks, no residual");
      const int Ho = H / 2, Wo = W / 2;
      constexpr int PC2 = (PH / 2) * 4;   // float4 per channel of the block's stride-2 output
#pragma unroll
      for (int i = 0; i < 16 * PC2 / NT; ++i) {
        const int idx = i * NT + tid;
        const int c = idx / PC2, q = idx % PC2;
        const int row = q >> 2, c4 = q & 3;
        const float* pp = plane_of(c) + (2 * row + 1) * 32 + 8 * c4 + 1;
        const int k = kb * w2::kNC + 16 * blk + c;
        const float bv = (EPI & 1) ? bias[k] : 0.0f;
        const size_t o = (((size_t)img * K + k) * Ho + y0 / 2 + row) * Wo + x0 / 2 + 4 * c4;
        const float4 v = make_float4(pp[0] + bv, pp[2] + bv, pp[4] + bv, pp[6] + bv);
        if (dbg & 128) __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(y + o));
        else if (!(dbg & 64)) *reinterpret_cast<float4*>(y + o) = v;
      }
      if (blk == 0) __syncthreads();
      continue;
    }
    // 16 channels × 1024 floats in 16-B chunks; a wave instruction = 1 KB of one channel:
    // TXB 8: 8 whole rows of the 32×32 block; TXB 4: one whole 16×16 image plane
    constexpr int PCF = TXB == 8 ? PH * 8 : NI * 64;   // float4 per channel plane
    constexpr int NIT = 16 * PCF / NT;                  // wave instructions per wave
    // TXB 8: wave w takes wave instructions 8w … 8w + 7 (1 KB = 8 rows of one channel each), so
    // each consecutive pair is one 16-row × 32-pixel segment of one channel: the GroupNorm
    // statistics below accumulate a pair in registers and reduce the wave's 4 segments together
    static_assert(TXB != 8 || NIT == 8, "TXB 8: eight wave instructions per wave");
    // (Σd, Σd²) of d = v − p around a pivot p per segment (a value of the segment: its first wave
    // instruction's lane-0 x), so a channel whose mean is far from 0 relative to its spread loses
    // nothing to cancellation; the segment leaves as (mean, M2) for Chan's combine (r05)
    float g1[4] = {0.f, 0.f, 0.f, 0.f}, g2[4] = {0.f, 0.f, 0.f, 0.f}, piv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int idx = TXB == 8 ? (((tid >> 6) * NIT + i) << 6) + (tid & 63) : i * NT + tid;
      const int c = idx / PCF, q = idx % PCF;
      const float4 v0 = *reinterpret_cast<const float4*>(plane_of(c) + 4 * q);
      const int k = kb * w2::kNC + 16 * blk + c;
      const float bv = (EPI & 1) ? bias[k] : 0.0f;
      size_t o;
      if (TXB == 8) {
        const int row = q >> 3, c4 = q & 7;
        o = (((size_t)img * K + k) * H + y0 + row) * W + x0 + 4 * c4;
      } else {
        o = ((size_t)(img + (q >> 6)) * K + k) * 256 + 4 * (q & 63);
      }
      float4 v = make_float4(v0.x + bv, v0.y + bv, v0.z + bv, v0.w + bv);
      if (EPI & 2) {
        const float4 rv = *reinterpret_cast<const float4*>(res + o);
        v.x += rv.x;
        v.y += rv.y;
        v.z += rv.z;
        v.w += rv.w;
      }
      if (dbg & 128) __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(y + o));
      else if (!(dbg & 64)) *reinterpret_cast<float4*>(y + o) = v;
      if (TXB == 8 && gnp) {   // the next GroupNorm's statistics: this lane's share of (Σd, Σd²)
        if ((i & 1) == 0) piv[i >> 1] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v.x)));
        const float p = piv[i >> 1];
        const float dx = v.x - p, dy = v.y - p, dz = v.z - p, dw = v.w - p;
        g1[i >> 1] += (dx + dy) + (dz + dw);
        g2[i >> 1] += (dx * dx + dy * dy) + (dz * dz + dw * dw);
      }
    }
    if (TXB == 8 && gnp) {
      // Reduce the wave's 8 values (Σ, Σ² of its 4 segments) over its 64 lanes together:
      // a permlane32 swap + add leaves 4 registers whose lane halves hold different values, a
      // permlane16 swap + add 2 whose 16-lane rows do, a row-mirror exchange 1 whose 8-lane
      // halves do; three DPP steps then finish each 8-lane group: group (row r, half h) = value
      // 2r + h, i.e. segment r's Σ (h 0) or Σ² (h 1).  (≈20 VALU instead of 8 full reductions.)
      float a[4] = {g1[0], g2[0], g1[1], g2[1]}, b[4] = {g1[2], g2[2], g1[3], g2[3]};
      float u[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a[j]), "+v"(b[j]));
        u[j] = a[j] + b[j];   // lanes 0-31: value j's partial, 32-63: value j + 4's
      }
      float w[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float x0 = u[j], x1 = u[j + 2];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x0), "+v"(x1));
        w[j] = x0 + x1;       // row r: value j + 2r
      }
      const int lane = tid & 63;
      const bool hi = (lane & 8) != 0;
      const float keep = hi ? w[1] : w[0], send = hi ? w[0] : w[1];
      float x = keep + dpp_read<0x140>(send);   // row_mirror: lane i <-> 15 - i
      x += dpp_read<0x141>(x);                  // row_half_mirror
      x += dpp_read<0x4E>(x);                   // quad_perm [2,3,0,1]
      x += dpp_read<0xB1>(x);                   // quad_perm [1,0,3,2]
      const float x2 = __shfl_xor(x, 8, 64);    // lane 16r: Σd of segment r, x2 its Σd²
      if ((lane & 15) == 0) {
        const int r = lane >> 4;
        const int J = (tid >> 6) * NIT + 2 * r;   // the segment's first wave instruction
        const int c = (J << 6) / PCF, piece = ((J << 6) % PCF) >> 6;
        const int k = kb * w2::kNC + 16 * blk + c;
        const int seg = ((y0 + 8 * piece) >> 4) * (W >> 5) + (x0 >> 5);
        const float p = r == 0 ? piv[0] : r == 1 ? piv[1] : r == 2 ? piv[2] : piv[3];
        constexpr float inv_n = 1.0f / 512.0f;   // 16 rows × 32 pixels
        gnp[((size_t)img * K + k) * (size_t)((H >> 4) * (W >> 5)) + seg] =
            make_float2(p + x * inv_n, fmaxf(x2 - x * (x * inv_n), 0.0f));
      }
    }
    if (blk == 0) __syncthreads();
  }
}

template <int EPI, int TXB, int NW = 8>
__global__ __launch_bounds__(NW * WAVE) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino2_kernel(
    const float* __restrict__ x, const float* __restrict__ U, const float* __restrict__ bias,
    const float* __restrict__ res, float* __restrict__ y, int nimg, int C, int K, int H, int W, int bw, int bpi,
    int nblk, int nkb, int kb_major, int csplit, int dbg, float2* __restrict__ gnp) {
  // separate LDS objects per ring slot: the compiler tells a DMA into one slot from a ds_read of
  // another and does not wait for outstanding DMAs before every LDS read
  __shared__ __attribute__((aligned(16))) float R0[w2::GeoT<TXB, NW>::RAWF], R1[w2::GeoT<TXB, NW>::RAWF],
      R2[(TXB == 4 && NW == 4) ? 4 : w2::GeoT<TXB, NW>::RAWF],
      R3[(TXB == 8 && NW == 8 && SKP_W2_RS4) ? w2::GeoT<TXB, NW>::RAWF : 4];
  __shared__ __attribute__((aligned(16))) float U0[w2::kUF], U1[w2::kUF], U2[NW == 4 ? 4 : w2::kUF];
  // workgroup → (input-channel split, 32×32-pixel block, channel block); consecutive logical ids
  // share one XCD.  A split sums its csplit input channels into slab sp of y (the workspace).
  const int G = gridDim.x;
  const int g = blockIdx.x;
  const int Lg = (G % 8 == 0) ? (g % 8) * (G / 8) + g / 8 : g;
  const int sp = Lg / (nblk * nkb);
  const int L = Lg - sp * (nblk * nkb);
  y += (size_t)sp * nimg * K * ((EPI & 4) ? (H / 2) * (W / 2) : H * W);   // EPI bit 2: stride-2 output
  int tb, kb;
  if (kb_major) {
    kb = L / nblk;
    tb = L - kb * nblk;
  } else {
    tb = L / nkb;
    kb = L - tb * nkb;
  }
  // TXB 8: block = 32×32 pixels of one image; TXB 4: images 4tb..4tb+3 whole
  int img, x0 = 0, y0 = 0;
  if (TXB == 8) {
    img = tb / bpi;
    const int br = tb - img * bpi;
    const int by = br / bw;
    x0 = 32 * (br - by * bw);
    y0 = (NW == 4 ? 16 : 32) * by;
  } else {
    img = (NW == 4 ? 2 : 4) * tb;
  }
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const W2Smem sm{R0, R1, R2, R3, U0, U1, U2};
  const int c0 = sp * csplit;
  if (wv < NW / 2)
    wino2_body<EPI, 0, TXB, NW>(sm, x, U, bias, res, y, C, K, H, W, img, x0, y0, kb, c0, csplit, wv, dbg, gnp);
  else wino2_body<EPI, 1, TXB, NW>(sm, x, U, bias, res, y, C, K, H, W, img, x0, y0, kb, c0, csplit, wv, dbg, gnp);
}

// U2[kb][c][k%32][40]: positions 0..17 at 0..17, 18..35 at 20..37, the rest zero
__global__ void wino2_weights_kernel(const float* __restrict__ w, int K, int C, int flip, float* __restrict__ U) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)K * C) return;
  const int k = (int)(i / C), c = (int)(i - (long long)k * C);
  double g[9];
  for (int u = 0; u < 3; ++u)
    for (int v = 0; v < 3; ++v)
      g[3 * u + v] = flip ? (double)w[((size_t)c * K + k) * 9 + (2 - u) * 3 + (2 - v)]
                          : (double)w[((size_t)k * C + c) * 9 + u * 3 + v];
  const double Gm[6][3] = {{1.0, 0.0, 0.0},
                           {1.0 / 3, 1.0 / 3, 1.0 / 3},
                           {-1.0 / 3, 1.0 / 3, -1.0 / 3},
                           {-16.0 / 15, -8.0 / 15, -4.0 / 15},
                           {1.0 / 15, -2.0 / 15, 4.0 / 15},
                           {0.0, 0.0, 1.0}};
  double t[6][3];
  for (int a = 0; a < 6; ++a)
    for (int v = 0; v < 3; ++v) t[a][v] = Gm[a][0] * g[v] + Gm[a][1] * g[3 + v] + Gm[a][2] * g[6 + v];
  float* out = U + (((size_t)(k / w2::kNC) * C + c) * w2::kNC + (k % w2::kNC)) * w2::kUP;
  for (int p = 0; p < w2::kUP; ++p) out[p] = 0.0f;
  for (int a = 0; a < 6; ++a)
    for (int b = 0; b < 6; ++b) {
      const int p = 6 * a + b;
      out[p < 18 ? p : p + 2] = (float)(t[a][0] * Gm[b][0] + t[a][1] * Gm[b][1] + t[a][2] * Gm[b][2]);
    }
}

}  // namespace

extern "C" int skp_wino2_weights(const float* w, int K, int C, int flip, float* U, void* stream) {
  SKP_CHECK_ARG(w && U, "null pointer");
  SKP_CHECK_ARG(K > 0 && C > 0, "non-positive shape");
  SKP_CHECK_ARG(K % w2::kNC == 0, "output channels must be a multiple of 32");
  const long long n = (long long)K * C;
  hipLaunchKernelGGL(wino2_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), w, K, C,
                     flip, U);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

// The VAE's Downsample2D (diffusers: F.pad(x, (0, 1, 0, 1)) then a 3×3 stride-2 convolution; reference
// ptp_utils.py:289-304 encodes through it): y[oy, ox] taps rows 2oy..2oy+2 and columns 2ox..2ox+2 with a
// zero row / column past the bottom-right edge, which is exactly the stride-1, pad-1 convolution sampled at
// the odd positions (2oy + 1, 2ox + 1).  The Winograd kernel computes the 32×32 blocks and its epilogue
// stores only the odd rows / columns (+ bias): no padded copy, no NCHW↔NHWC transposes, no bias pass.
namespace {
// flag 128 of the kernels' flag word: non-temporal output stores, for outputs of at least 256 MB
// (larger than the Infinity Cache: the next layer re-reads them from HBM either way, and the stream
// then does not evict the input regions / weights the other workgroups re-read from L2)
int wino_nt_flag(long long out_bytes, int nsplit) {
  if (nsplit > 1) return 0;   // split-K partials are re-read by the reduction
  return out_bytes >= (256LL << 20) ? 128 : 0;
}
}  // namespace

extern "C" int skp_conv3x3s2_wino2(const float* x, const float* U, const float* bias, float* y, int B, int C, int K,
                                   int H, int W, int nsplit, float* ws, void* stream) {
  SKP_CHECK_ARG(x && U && y, "null pointer");
  SKP_CHECK_ARG(B > 0 && C > 0 && K > 0 && H > 0 && W > 0, "non-positive shape");
  SKP_CHECK_ARG(C % w2::kCK == 0, "input channels must be a multiple of 4");
  SKP_CHECK_ARG(K % w2::kNC == 0, "output channels must be a multiple of 32");
  SKP_CHECK_ARG(H % 32 == 0 && W % 32 == 0, "H and W must be multiples of 32");
  SKP_CHECK_ARG(nsplit >= 1 && C % (w2::kCK * nsplit) == 0, "nsplit must divide C into multiples of 4");
  SKP_CHECK_ARG(nsplit == 1 || ws, "split-K needs a workspace of nsplit·B·K·(H/2)·(W/2) floats");
  SKP_CHECK_ARG(aligned16(x) && aligned16(U) && aligned16(y) && (!ws || aligned16(ws)), "tensors must be 16-byte aligned");
  SKP_CHECK_ARG((long long)B * C * H * W * 4 < 0x7fffffffLL, "input larger than 2 GiB (32-bit buffer offsets)");
  // half-height blocks (see skp_conv3x3_wino2)
  const int bw = W / 32, bpi = (H / 16) * bw;
  const long long nblk = (long long)B * bpi;
  const int nkb = K / w2::kNC;
  SKP_CHECK_ARG(nblk * nkb * nsplit <= 0x7fffffffLL, "grid too large");
  float* out = nsplit > 1 ? ws : y;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(nblk * nkb * nsplit));
  const int fl = SKP_WINO2_DEBUG | wino_nt_flag((long long)B * K * (H / 2) * (W / 2) * 4, nsplit);
  if (nsplit == 1 && bias)
    hipLaunchKernelGGL((wino2_kernel<5, 8, 4>), grid, dim3(4 * WAVE), 0, st, x, U, bias, nullptr, out, B, C, K, H, W,
                       bw, bpi, (int)nblk, nkb, 0, C / nsplit, fl, nullptr);
  else
    hipLaunchKernelGGL((wino2_kernel<4, 8, 4>), grid, dim3(4 * WAVE), 0, st, x, U, nullptr, nullptr, out, B, C, K, H,
                       W, bw, bpi, (int)nblk, nkb, 0, C / nsplit, fl, nullptr);
  SKP_LAUNCH_CHECK();
  if (nsplit > 1) return splitk_reduce(ws, nsplit, B, K, (H / 2) * (W / 2), bias, nullptr, y, st);
  return SKP_OK;
}

extern "C" int skp_conv3x3_wino2_gn(const float* x, const float* U, const float* bias, const float* residual, float* y,
                                    int B, int C, int K, int H, int W, int nsplit, float* ws, float* gn_part,
                                    void* stream) {
  SKP_CHECK_ARG(x && U && y, "null pointer");
  SKP_CHECK_ARG(!gn_part || (nsplit == 1 && H % 32 == 0 && W % 32 == 0 && (reinterpret_cast<uintptr_t>(gn_part) & 7) == 0),
                "gn_part: one split, H and W multiples of 32, 8-byte aligned");
  SKP_CHECK_ARG(B > 0 && C > 0 && K > 0 && H > 0 && W > 0, "non-positive shape");
  SKP_CHECK_ARG(C % w2::kCK == 0, "input channels must be a multiple of 4");
  SKP_CHECK_ARG(K % w2::kNC == 0, "output channels must be a multiple of 32");
  const bool g16 = H == 16 && W == 16;
  SKP_CHECK_ARG((H % 32 == 0 && W % 32 == 0) || (g16 && B % 4 == 0),
                "H and W must be multiples of 32, or 16×16 with B a multiple of 4");
  SKP_CHECK_ARG(nsplit >= 1 && C % (w2::kCK * nsplit) == 0, "nsplit must divide C into multiples of 4");
  SKP_CHECK_ARG(nsplit == 1 || ws, "split-K needs a workspace of nsplit·B·K·H·W floats");
  SKP_CHECK_ARG(aligned16(x) && aligned16(U) && aligned16(y) && (!residual || aligned16(residual)) &&
                    (!ws || aligned16(ws)),
                "tensors must be 16-byte aligned");
  SKP_CHECK_ARG((long long)B * C * H * W * 4 < 0x7fffffffLL, "input larger than 2 GiB (32-bit buffer offsets)");
  // half-height blocks (32 × 16 pixels, 4 waves, two workgroups per CU: one's prologue / epilogue
  // overlaps the other's stage loop), 5-11% faster than the 32 × 32 one-workgroup-per-CU form at
  // every VAE / UNet shape (profiles/r03al_wino_half_ab.txt); the 16×16 geometry as two images per
  // 4-wave workgroup, two workgroups per CU (profiles/r03ap_wino_half16_ab.txt)
  const int bw = W / 32, bpi = (H / 16) * bw;
  const long long nblk = g16 ? B / 2 : (long long)B * bpi;
  const int nkb = K / w2::kNC;
  SKP_CHECK_ARG(nblk * nkb * nsplit <= 0x7fffffffLL, "grid too large");
  const int dbg = SKP_WINO2_DEBUG;
  // tile-major (the channel blocks of one pixel block back to back, sharing its input region in
  // L2) measured 1-2% ahead of channel-block-major at every VAE / UNet shape, U size regardless
  const int kb_major = 0;
  const int epi = nsplit > 1 ? 0 : (bias ? 1 : 0) | (residual ? 2 : 0);
  float* out = nsplit > 1 ? ws : y;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(nblk * nkb * nsplit));
  const int fl = dbg | wino_nt_flag((long long)B * K * H * W * 4, nsplit);
  float2* gnp = reinterpret_cast<float2*>(gn_part);
#define SKP_WG2(E)                                                                                            \
  if (g16)                                                                                                    \
    hipLaunchKernelGGL((wino2_kernel<E, 4, 4>), grid, dim3(4 * WAVE), 0, st, x, U, bias, residual, out, B, C, K,  \
                       H, W, bw, bpi, (int)nblk, nkb, kb_major, C / nsplit, fl, nullptr);                              \
  else                                                                                                        \
    hipLaunchKernelGGL((wino2_kernel<E, 8, 4>), grid, dim3(4 * WAVE), 0, st, x, U, bias, residual, out, B, C, K,  \
                       H, W, bw, bpi, (int)nblk, nkb, kb_major, C / nsplit, fl, gnp)
  switch (epi) {
    case 0: SKP_WG2(0); break;
    case 1: SKP_WG2(1); break;
    case 2: SKP_WG2(2); break;
    default: SKP_WG2(3); break;
  }
#undef SKP_WG2
  SKP_LAUNCH_CHECK();
  if (nsplit > 1) return splitk_reduce(ws, nsplit, B, K, H * W, bias, residual, y, st);
  return SKP_OK;
}

extern "C" int skp_conv3x3_wino2(const float* x, const float* U, const float* bias, const float* residual, float* y,
                                 int B, int C, int K, int H, int W, int nsplit, float* ws, void* stream) {
  return skp_conv3x3_wino2_gn(x, U, bias, residual, y, B, C, K, H, W, nsplit, ws, nullptr, stream);
}
