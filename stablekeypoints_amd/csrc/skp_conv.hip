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

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kMT = 64;                       // output tiles per workgroup
constexpr int kNC = 32;                       // output channels per workgroup
constexpr int kCK = 4;                        // input channels per LDS stage (= MFMA k)
constexpr int kP = 36;                        // transform positions (6×6)
constexpr int kThreads = 512;                 // 8 waves, two per SIMD
constexpr int kVs = kCK * kMT * kP;           // floats per V stage  (9216)
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
__device__ __forceinline__ void transform_patch(const char* raw, unsigned mask, int lane, float* vd) {
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
    *reinterpret_cast<float2*>(vd + 6 * i) = make_float2(v[0], v[1]);
    *reinterpret_cast<float2*>(vd + 6 * i + 2) = make_float2(v[2], v[3]);
    *reinterpret_cast<float2*>(vd + 6 * i + 4) = make_float2(v[4], v[5]);
  }
}

// EPI bit 0: + bias[k]; bit 1: + residual (same layout as y)
template <int EPI>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_f4_kernel(
    const float* __restrict__ x, const float* __restrict__ U, const float* __restrict__ bias,
    const float* __restrict__ res, float* __restrict__ y, int nimg, int C, int K, int H, int W, int tw, int tpi,
    int ntiles, int ntb, int nkb, int kb_major, int dbg) {
  // separate LDS objects per buffer, so the compiler can tell a DMA into one buffer from a
  // ds_read of another and does not wait for the DMA before every LDS read
  __shared__ __attribute__((aligned(16))) float V0[kVs], V1[kVs];   // [kCK][kMT][kP]
  __shared__ __attribute__((aligned(16))) float U0[kUs], U1[kUs];   // [kCK][kNC][kP]
  __shared__ __attribute__((aligned(16))) char Raw[4 * kRawWave];   // [4 waves][6 rows][mid | left | right]

  // workgroup → (tile block, channel block); consecutive logical ids share one XCD
  const int G = gridDim.x;
  const int g = blockIdx.x;
  const int L = (G % 8 == 0) ? (g % 8) * (G / 8) + g / 8 : g;
  int tb, kb;
  if (kb_major) {
    kb = L / ntb;
    tb = L - kb * ntb;
  } else {
    tb = L / nkb;
    kb = L - tb * nkb;
  }

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv & 3, wn = wv >> 2;   // this wave's 16 tiles × 16 channels
  const bool patcher = wv < 4;            // waves 0-3: patches of stage channel wv; 4-7: U slices
  const size_t plane = (size_t)H * W;
  PatchAddr pa;
  {
    const int pt = tb * kMT + lane;
    const bool pvalid = pt < ntiles;
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
  const float* Ub = U + (size_t)kb * C * kNC * kP;
  const int nst = C / kCK;
  const size_t xfloats = (size_t)nimg * C * plane;
  char* raw = Raw + (wv & 3) * kRawWave;
  const int vrow = ((wv & 3) * kMT + lane) * kP;   // this patcher lane's V row
  // per-stage descriptors: x from the stage's first channel plane, U from the stage's slice
  auto xrsrc = [&](int s) {
    const size_t off = (size_t)s * kCK * plane;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(x + off), (short)0, (dbg & 1) ? 0 : (int)((xfloats - off) * 4), 0x00020000);
  };
  auto dma_u = [&](int s, float* ubuf) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(Ub + (size_t)s * kUs), (short)0, (dbg & 2) ? 0 : kUs * 4, 0x00020000);
    char* dst = reinterpret_cast<char*>(ubuf);
#pragma unroll
    for (int c = wv - 4; c < kUChunks; c += 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + c * 1024), 16, lane * 16, c * 1024, 0, 0);
  };

  f32x4 acc[kP];
#pragma unroll
  for (int p = 0; p < kP; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: V[0] and U[0] ready, stage 1's raw patches in flight
  if (patcher) {
    dma_patches(xrsrc(0), pa, raw);
    __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) & lgkmcnt(0): this wave's DMA landed
    transform_patch(raw, pa.mask, lane, V0 + vrow);
    if (nst > 1) dma_patches(xrsrc(1), pa, raw);
  } else {
    dma_u(0, U0);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  // MFMA operands: A = V[k = lane>>4][tile 16·wm + (lane&15)], B = U[k][channel 16·wn + (lane&15)]
  const int aoff = ((lane >> 4) * kMT + wm * 16 + (lane & 15)) * kP;
  const int boff = ((lane >> 4) * kNC + wn * 16 + (lane & 15)) * kP;
  // one stage: prepare stage s+1 into (vn, un), MFMAs on (vc, uc); the loop is unrolled by two
  // so every buffer is a fixed LDS object in each half
  auto phase = [&](int s, const float* vc, const float* uc, float* vn, float* un) {
    if (s + 1 < nst) {
      if (patcher) {
        transform_patch(raw, pa.mask, lane, vn + vrow);
        if (s + 2 < nst) dma_patches(xrsrc(s + 2), pa, raw);
      } else {
        dma_u(s + 1, un);
      }
    }
    const float* va = vc + aoff;
    const float* ub = uc + boff;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
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
  const int k = kb * kNC + wn * 16 + (lane & 15);
  const float bv = (EPI & 1) ? bias[k] : 0.0f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int t = tb * kMT + wm * 16 + 4 * (lane >> 4) + r;
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

extern "C" int skp_conv3x3_wino(const float* x, const float* U, const float* bias, const float* residual, float* y,
                                int B, int C, int K, int H, int W, void* stream) {
  SKP_CHECK_ARG(x && U && y, "null pointer");
  SKP_CHECK_ARG(B > 0 && C > 0 && K > 0 && H > 0 && W > 0, "non-positive shape");
  SKP_CHECK_ARG(C % kCK == 0, "input channels must be a multiple of 4");
  SKP_CHECK_ARG(K % kNC == 0, "output channels must be a multiple of 32");
  SKP_CHECK_ARG(H % 4 == 0 && W % 4 == 0, "H and W must be multiples of 4");
  SKP_CHECK_ARG(aligned16(x) && aligned16(U) && aligned16(y) && (!residual || aligned16(residual)),
                "tensors must be 16-byte aligned");
  const int tw = W / 4, tpi = (H / 4) * tw;
  const long long ntiles = (long long)B * tpi;
  SKP_CHECK_ARG(ntiles <= 0x7fffffffLL - kMT, "too many tiles");
  SKP_CHECK_ARG((long long)B * C * H * W * 4 < 0x7fffffffLL, "input larger than 2 GiB (32-bit buffer offsets)");
  const int ntb = (int)((ntiles + kMT - 1) / kMT), nkb = K / kNC;
  SKP_CHECK_ARG((long long)ntb * nkb <= 0x7fffffffLL, "grid too large");
  // one channel block's U slice is C·32·36·4 B; keep all of U on an L2 slice when it fits
  const long long ubytes = (long long)K * C * kP * 4;
  const int kb_major = ubytes > (2LL << 20);
  const int epi = (bias ? 1 : 0) | (residual ? 2 : 0);
  static const int dbg = getenv("SKP_WINO_DEBUG") ? atoi(getenv("SKP_WINO_DEBUG")) : 0;   // dev: 1 drop x loads, 2 drop U loads
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(ntb * nkb));
#define SKP_WG(E)                                                                                                 \
  hipLaunchKernelGGL((wino_f4_kernel<E>), grid, dim3(kThreads), 0, st, x, U, bias, residual, y, B, C, K, H, W, \
                     tw, tpi, (int)ntiles, ntb, nkb, kb_major, dbg)
  switch (epi) {
    case 0: SKP_WG(0); break;
    case 1: SKP_WG(1); break;
    case 2: SKP_WG(2); break;
    default: SKP_WG(3); break;
  }
#undef SKP_WG
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
