// UNet-side: fused softmax backward of the frozen UNet's attention (diffusers-0.8.0
// CrossAttention, the math path softmax(q kᵀ·scale) v) on gfx950.
//
// For each row of P = softmax(S) and its gradient dP:  dS = alpha · P ⊙ (dP − Σ_j P_j dP_j),
// written over dP.  PyTorch runs this as a product pass, a reduction pass and the scale
// multiply of baddbmm's backward (three passes over the 64²-token layers' (B·H, 4096, 4096)
// fp32 tensors, 4.3 GB each at batch 8); here it is one read of P and dP and one write.
// A row is owned by one wave (≤ 1024 columns) or one 256 / 1024-thread workgroup and stays in
// registers between the reduction and the update.
#include "skp_common.h"

using namespace skp;

namespace {

template <int TPR, int EPT, bool VEC>   // threads per row, elements per thread, float4 path (EPT % 4 == 0)
__global__ __launch_bounds__(TPR) void softmax_bwd_kernel(const float* __restrict__ P, float* __restrict__ G,
                                                          long long rows, int cols, float alpha) {
  __shared__ float sred[TPR / WAVE];
  const long long row = blockIdx.x;
  if (row >= rows) return;
  const float* p = P + row * cols;
  float* g = G + row * cols;
  static_assert(!VEC || EPT % 4 == 0, "float4 path needs EPT % 4 == 0");
  float pv[EPT], gv[EPT];
  float dot = 0.0f;
  if (VEC) {
#pragma unroll
    for (int q = 0; q < EPT / 4; ++q) {
      const int e = 4 * (threadIdx.x + q * TPR);
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (e < cols) {
        a = *reinterpret_cast<const float4*>(p + e);
        b = *reinterpret_cast<const float4*>(g + e);
      }
      pv[4 * q] = a.x; pv[4 * q + 1] = a.y; pv[4 * q + 2] = a.z; pv[4 * q + 3] = a.w;
      gv[4 * q] = b.x; gv[4 * q + 1] = b.y; gv[4 * q + 2] = b.z; gv[4 * q + 3] = b.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = threadIdx.x + q * TPR;
      pv[q] = e < cols ? p[e] : 0.0f;
      gv[q] = e < cols ? g[e] : 0.0f;
    }
  }
#pragma unroll
  for (int q = 0; q < EPT; ++q) dot += pv[q] * gv[q];
  dot = wave_sum(dot);
  if (TPR > WAVE) {
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    if (lane == 0) sred[wid] = dot;
    __syncthreads();
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < TPR / WAVE; ++w) t += sred[w];
    dot = t;
  }
  if (VEC) {
#pragma unroll
    for (int q = 0; q < EPT / 4; ++q) {
      const int e = 4 * (threadIdx.x + q * TPR);
      if (e < cols)
        *reinterpret_cast<float4*>(g + e) =
            make_float4(alpha * (pv[4 * q] * (gv[4 * q] - dot)), alpha * (pv[4 * q + 1] * (gv[4 * q + 1] - dot)),
                        alpha * (pv[4 * q + 2] * (gv[4 * q + 2] - dot)),
                        alpha * (pv[4 * q + 3] * (gv[4 * q + 3] - dot)));
    }
  } else {
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = threadIdx.x + q * TPR;
      if (e < cols) g[e] = alpha * (pv[q] * (gv[q] - dot));
    }
  }
}

// In-place row softmax, torch order: m = max, e = exp(x − m), y = e / Σe.  A row stays in
// registers between the two reductions: one read and one write of S.
template <int TPR, int EPT>   // float4 lanes: EPT % 4 == 0
__global__ __launch_bounds__(TPR) void softmax_fwd_kernel(float* __restrict__ S, long long rows, int cols) {
  __shared__ float sred[2][TPR / WAVE];
  const long long row = blockIdx.x;
  if (row >= rows) return;
  float* p = S + row * cols;
  float v[EPT];
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < EPT / 4; ++q) {
    const int e = 4 * (threadIdx.x + q * TPR);
    float4 a = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    if (e < cols) a = *reinterpret_cast<const float4*>(p + e);
    v[4 * q] = a.x;
    v[4 * q + 1] = a.y;
    v[4 * q + 2] = a.z;
    v[4 * q + 3] = a.w;
    m = fmaxf(m, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
  }
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  m = wave_max(m);
  if (TPR > WAVE) {
    if (lane == 0) sred[0][wid] = m;
    __syncthreads();
    float t = sred[0][0];
#pragma unroll
    for (int w = 1; w < TPR / WAVE; ++w) t = fmaxf(t, sred[0][w]);
    m = t;
  }
  float sum = 0.0f;
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    v[q] = expf(v[q] - m);
    sum += v[q];
  }
  sum = wave_sum(sum);
  if (TPR > WAVE) {
    if (lane == 0) sred[1][wid] = sum;
    __syncthreads();
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < TPR / WAVE; ++w) t += sred[1][w];
    sum = t;
  }
#pragma unroll
  for (int q = 0; q < EPT / 4; ++q) {
    const int e = 4 * (threadIdx.x + q * TPR);
    if (e < cols)
      *reinterpret_cast<float4*>(p + e) =
          make_float4(v[4 * q] / sum, v[4 * q + 1] / sum, v[4 * q + 2] / sum, v[4 * q + 3] / sum);
  }
}

}  // namespace

extern "C" int skp_softmax_fwd(float* S, long long rows, int cols, void* stream) {
  SKP_CHECK_ARG(S, "null pointer");
  SKP_CHECK_ARG(rows > 0 && cols > 0, "non-positive shape");
  SKP_CHECK_ARG(cols <= 16384 && cols % 4 == 0, "cols must be a multiple of 4, at most 16384");
  SKP_CHECK_ARG(rows <= 0x7fffffffLL, "too many rows");
  SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(S) & 15) == 0, "S must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)rows);
#define SKP_SF(T, E) hipLaunchKernelGGL((softmax_fwd_kernel<T, E>), grid, dim3(T), 0, st, S, rows, cols)
  if (cols <= 64 * 4) SKP_SF(64, 4);
  else if (cols <= 64 * 8) SKP_SF(64, 8);
  else if (cols <= 64 * 16) SKP_SF(64, 16);
  else if (cols <= 256 * 16) SKP_SF(256, 16);
  else SKP_SF(1024, 16);
#undef SKP_SF
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_softmax_bwd(const float* P, float* dP, long long rows, int cols, float alpha, void* stream) {
  SKP_CHECK_ARG(P && dP, "null pointer");
  SKP_CHECK_ARG(rows > 0 && cols > 0, "non-positive shape");
  SKP_CHECK_ARG(cols <= 16384, "rows longer than 16384 are not supported");
  SKP_CHECK_ARG(rows <= 0x7fffffffLL, "too many rows");
  const bool aligned = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(dP)) & 15) == 0;
  const bool vec = aligned && (cols % 4 == 0);
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)rows);
#define SKP_SB(T, E, V) \
  hipLaunchKernelGGL((softmax_bwd_kernel<T, E, V>), grid, dim3(T), 0, st, P, dP, rows, cols, alpha)
  if (vec) {   // float4 per lane: up to 16 elements per thread
    if (cols <= 64 * 4) SKP_SB(64, 4, true);
    else if (cols <= 64 * 8) SKP_SB(64, 8, true);
    else if (cols <= 64 * 16) SKP_SB(64, 16, true);
    else if (cols <= 256 * 16) SKP_SB(256, 16, true);
    else SKP_SB(1024, 16, true);
  } else {
    if (cols <= 64 * 2) SKP_SB(64, 2, false);
    else if (cols <= 64 * 8) SKP_SB(64, 8, false);
    else if (cols <= 64 * 16) SKP_SB(64, 16, false);
    else if (cols <= 256 * 16) SKP_SB(256, 16, false);
    else SKP_SB(1024, 16, false);
  }
#undef SKP_SB
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

// ------------------------------------------------------------------------------------------------
// Fused attention score gradient (diffusers math attention backward, the 4096-token layers):
//   dS = alpha · P ⊙ (dO·Vᵀ − D),   D[row] = Σ_j P_row,j (dO·Vᵀ)_row,j = dO_row · O_row
// dP = dO·Vᵀ is computed on the fly on the f32 matrix cores (K = the head dim) instead of being
// written and re-read as a (B·H, S, L) tensor, and D comes from the forward output (the flash-
// attention identity), so one pass reads P once and writes dS once (over P when out == P).
// Workgroup = 64 keys × 64 rows of one head, 4 waves.  The dO and V tiles are staged in LDS
// (16-B global loads, rows padded to d+1 floats: conflict-free operand reads); wave w computes
// dPᵀ for keys 16w..16w+15 × the four 16-row blocks with four independent accumulators, so each
// lane ends with 4 consecutive keys of one row: P is read and dS written as float4.
namespace {
typedef float f32x4a __attribute__((ext_vector_type(4)));

template <int KS>   // head dim / 4
__global__ __launch_bounds__(256) void attn_dscore_kernel(const float* P, const float* __restrict__ dO,
                                                          const float* __restrict__ V, const float* __restrict__ D,
                                                          float* out, int S, int L, float alpha) {
  constexpr int d = 4 * KS, dp = d + 1;
  __shared__ float sO[64 * dp], sV[64 * dp];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 64, k0 = blockIdx.x * 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  {
    const float4* gO = reinterpret_cast<const float4*>(dO + ((size_t)b * S + r0) * d);
    const float4* gV = reinterpret_cast<const float4*>(V + ((size_t)b * L + k0) * d);
    for (int e = t; e < 64 * KS; e += 256) {
      const int row = e / KS, c = 4 * (e - row * KS);
      const float4 o = gO[e], v = gV[e];
      float* po = sO + row * dp + c;
      float* pv = sV + row * dp + c;
      po[0] = o.x; po[1] = o.y; po[2] = o.z; po[3] = o.w;
      pv[0] = v.x; pv[1] = v.y; pv[2] = v.z; pv[3] = v.w;
    }
  }
  __syncthreads();
  // A = V rows (keys 16w + (lane&15)), B = dO rows (16bj + (lane&15)); k = 4ks + (lane>>4)
  const float* va = sV + (16 * w + (lane & 15)) * dp + (lane >> 4);
  const float* ob = sO + (lane & 15) * dp + (lane >> 4);
  f32x4a acc[4];
#pragma unroll
  for (int bj = 0; bj < 4; ++bj) acc[bj] = f32x4a{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const float a = va[4 * ks];
#pragma unroll
    for (int bj = 0; bj < 4; ++bj)
      acc[bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ob[16 * bj * dp + 4 * ks], acc[bj], 0, 0, 0);
  }
  // lane: keys k0 + 16w + 4(lane>>4) .. +3 of row r0 + 16bj + (lane&15)
  const int key = k0 + 16 * w + 4 * (lane >> 4);
#pragma unroll
  for (int bj = 0; bj < 4; ++bj) {
    const int row = r0 + 16 * bj + (lane & 15);
    const float dr = D[(size_t)b * S + row];
    const size_t o = ((size_t)b * S + row) * L + key;
    const float4 p = *reinterpret_cast<const float4*>(P + o);
    *reinterpret_cast<float4*>(out + o) =
        make_float4(alpha * (p.x * (acc[bj][0] - dr)), alpha * (p.y * (acc[bj][1] - dr)),
                    alpha * (p.z * (acc[bj][2] - dr)), alpha * (p.w * (acc[bj][3] - dr)));
  }
}
}  // namespace

extern "C" int skp_attn_dscore(const float* P, const float* dO, const float* V, const float* D, float* out, int BH,
                               int S, int L, int d, float alpha, void* stream) {
  SKP_CHECK_ARG(P && dO && V && D && out, "null pointer");
  SKP_CHECK_ARG(BH > 0 && S > 0 && L > 0 && d > 0, "non-positive shape");
  SKP_CHECK_ARG(S % 64 == 0 && L % 64 == 0, "S and L must be multiples of 64");
  SKP_CHECK_ARG(((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(dO) | reinterpret_cast<uintptr_t>(V) |
                  reinterpret_cast<uintptr_t>(out)) & 15) == 0,
                "tensors must be 16-byte aligned");
  SKP_CHECK_ARG(BH <= 65535 && S / 64 <= 65535, "grid too large");
  const dim3 grid((unsigned)(L / 64), (unsigned)(S / 64), (unsigned)BH);
  hipStream_t st = as_stream(stream);
#define SKP_DS(K) hipLaunchKernelGGL((attn_dscore_kernel<K>), grid, dim3(256), 0, st, P, dO, V, D, out, S, L, alpha)
  switch (d) {
    case 40: SKP_DS(10); break;
    case 64: SKP_DS(16); break;
    case 80: SKP_DS(20); break;
    case 160: SKP_DS(40); break;
    default: SKP_CHECK_ARG(false, "head dim must be 40, 64, 80 or 160");
  }
#undef SKP_DS
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

// ------------------------------------------------------------------------------------------------
// Head layouts of the attention operands.  Row s of head b·H + h starts at base + b·sb + h·d + s·rs:
//   (B·H, S, d) contiguous:               H = 1, sb = S·d, rs = d;
//   (B, S, H·d), the projections' own layout (diffusers' to_q / to_k / to_v output and to_out
//   input, no head permute):             sb = S·H·d, rs = H·d;
//   a context shared by the batch (the token embedding expanded over B): sb = 0.
struct AttnLay {
  long long sb;
  int rs;
  template <typename T>
  __device__ __forceinline__ T* at(T* base, int bh, int H, int d) const {
    const int b = bh / H;
    return base + (size_t)b * sb + (size_t)(bh - b * H) * d;
  }
};

// ------------------------------------------------------------------------------------------------
// Forward-only fused attention O = softmax(scale·Q Kᵀ) V for the UNet's self-attention layers
// that need no backward (the first 64²-token layer: its input does not depend on the token
// embedding), so no (B·H, S, L) score or probability tensor is written or read.
// Workgroup = 64 query rows of one head, 4 waves (16 rows each), looping over 64-key blocks:
//   Sᵀ = K·Qᵀ on the f32 matrix cores (lane: 4 consecutive keys × 1 query row of each 16-key
//   sub-block), online row max / sum (a row's 64 keys live in 4 lanes: two xor-shuffles), then
//   Oᵀ += Vᵀ·Pᵀ with the same (permuted) key order as the k dimension — the C layout of Sᵀ is
//   the B operand as it stands, no transposition.  K / V tiles are staged in LDS (16-B loads).
namespace {

template <int KS, int DB>   // head dim / 4, 16-wide head-dim blocks (d ≤ 16·DB)
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                       const float* __restrict__ V, float* __restrict__ O,
                                                       float2* __restrict__ ST, int S, int L, float scale, int H,
                                                       AttnLay lq, AttnLay lk, AttnLay lv, AttnLay lo) {
  constexpr int d = 4 * KS, dp = d + 1;
  __shared__ float sK[64 * dp], sV[64 * 16 * DB];   // sV rows padded to 16·DB with zeros
  const int b = blockIdx.y;                         // b·H + h
  const int r0 = blockIdx.x * 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int row = r0 + 16 * w + (lane & 15);        // this lane's query row
  const float* Qb = lq.at(Q, b, H, d);
  const float* Kb = lk.at(K, b, H, d);
  const float* Vb = lv.at(V, b, H, d);
  // B operand of Sᵀ = K·Qᵀ: Qᵀ[k = 4ks + (lane>>4)][j = row] (pre-scaled)
  float qv[KS];
  {
    const float* q = Qb + (size_t)row * lq.rs + (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qv[ks] = q[4 * ks] * scale;
  }
  f32x4a o[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db) o[db] = f32x4a{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.0f;
  for (int k0 = 0; k0 < L; k0 += 64) {
    __syncthreads();   // previous block's tiles consumed
    {
      for (int e = t; e < 64 * KS; e += 256) {
        const int key = e / KS, c = 4 * (e - key * KS);
        float4 kk = make_float4(0.f, 0.f, 0.f, 0.f), vv = kk;   // keys past L (ragged last block): zero
        if (k0 + key < L) {
          kk = *reinterpret_cast<const float4*>(Kb + (size_t)(k0 + key) * lk.rs + c);
          vv = *reinterpret_cast<const float4*>(Vb + (size_t)(k0 + key) * lv.rs + c);
        }
        float* pk = sK + key * dp + c;
        pk[0] = kk.x; pk[1] = kk.y; pk[2] = kk.z; pk[3] = kk.w;
        *reinterpret_cast<float4*>(sV + key * 16 * DB + c) = vv;
      }
      if constexpr (16 * DB > d)
        for (int e = t; e < 64 * (16 * DB - d); e += 256) {
          const int key = e / (16 * DB - d), c = d + (e - key * (16 * DB - d));
          sV[key * 16 * DB + c] = 0.0f;
        }
    }
    __syncthreads();
    // Sᵀ sub-blocks c: lane holds keys 16c + 4(lane>>4) + r, row (lane & 15)
    f32x4a s4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      s4[c] = f32x4a{0.f, 0.f, 0.f, 0.f};
      const float* kr = sK + (16 * c + (lane & 15)) * dp + (lane >> 4);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) s4[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(kr[4 * ks], qv[ks], s4[c], 0, 0, 0);
    }
    if (k0 + 64 > L) {   // keys past L take no probability
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (k0 + 16 * c + 4 * (lane >> 4) + r >= L) s4[c][r] = -INFINITY;
    }
    float bm = -INFINITY;
#pragma unroll
    for (int c = 0; c < 4; ++c) bm = fmaxf(bm, fmaxf(fmaxf(s4[c][0], s4[c][1]), fmaxf(s4[c][2], s4[c][3])));
    bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
    bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
    const float mn = fmaxf(m, bm);
    const float corr = __expf(m - mn);   // 0 on the first block (m = -inf)
    float bs = 0.0f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s4[c][r] = __expf(s4[c][r] - mn);
        bs += s4[c][r];
      }
    bs += __shfl_xor(bs, 16, 64);
    bs += __shfl_xor(bs, 32, 64);
    l = l * corr + bs;
    m = mn;
#pragma unroll
    for (int db = 0; db < DB; ++db) o[db] *= corr;
    // Oᵀ[d][row] += Σ_key V[key][d] · P[key][row]; k-step (c, r) covers keys 16c + 4(lane>>4) + r
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float* vr = sV + (16 * c + 4 * (lane >> 4) + r) * 16 * DB + (lane & 15);
#pragma unroll
        for (int db = 0; db < DB; ++db)
          o[db] = __builtin_amdgcn_mfma_f32_16x16x4f32(vr[16 * db], s4[c][r], o[db], 0, 0, 0);
      }
  }
  // lane: Oᵀ[d = 16db + 4(lane>>4) + r][row (lane & 15)] → O[row][d..d+3]
  const float inv = 1.0f / l;
  float* orow = lo.at(O, b, H, d) + (size_t)row * lo.rs;
#pragma unroll
  for (int db = 0; db < DB; ++db) {
    const int dd = 16 * db + 4 * (lane >> 4);
    if (dd < d) *reinterpret_cast<float4*>(orow + dd) = make_float4(o[db][0] * inv, o[db][1] * inv, o[db][2] * inv, o[db][3] * inv);
  }
  // row stats for a backward that recomputes P = exp(scale·q·k − m) / l (the 4 lanes of a row agree)
  if (ST != nullptr && lane < 16) ST[(size_t)b * S + row] = make_float2(m, inv);
}

}  // namespace

namespace {
int attn_fwd_launch(const float* Q, AttnLay lq, const float* K, AttnLay lk, const float* V, AttnLay lv, float* O,
                    AttnLay lo, float* stats, int BH, int H, int S, int L, int d, float scale, void* stream) {
  SKP_CHECK_ARG(Q && K && V && O, "null pointer");
  SKP_CHECK_ARG(BH > 0 && H > 0 && BH % H == 0 && S > 0 && L > 0, "non-positive shape");
  SKP_CHECK_ARG(S % 64 == 0, "S must be a multiple of 64");
  SKP_CHECK_ARG(BH <= 65535, "grid too large");
  SKP_CHECK_ARG(((reinterpret_cast<uintptr_t>(K) | reinterpret_cast<uintptr_t>(V) | reinterpret_cast<uintptr_t>(O)) &
                 15) == 0,
                "tensors must be 16-byte aligned");
  SKP_CHECK_ARG(((lk.rs | lv.rs | lo.rs | lk.sb | lv.sb | lo.sb) & 3) == 0, "K, V, O strides must be multiples of 4");
  SKP_CHECK_ARG((reinterpret_cast<uintptr_t>(stats) & 7) == 0, "stats must be 8-byte aligned");
  const dim3 grid((unsigned)(S / 64), (unsigned)BH);
  hipStream_t st = as_stream(stream);
  float2* ST = reinterpret_cast<float2*>(stats);
#define SKP_AF(KS_, DB_)                                                                                        \
  hipLaunchKernelGGL((attn_fwd_kernel<KS_, DB_>), grid, dim3(256), 0, st, Q, K, V, O, ST, S, L, scale, H, lq, lk, lv, \
                     lo)
  switch (d) {
    case 40: SKP_AF(10, 3); break;
    case 64: SKP_AF(16, 4); break;
    case 80: SKP_AF(20, 5); break;
    default: SKP_CHECK_ARG(false, "head dim must be 40, 64 or 80");
  }
#undef SKP_AF
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
AttnLay contig(int rows, int d) { return AttnLay{(long long)rows * d, d}; }
}  // namespace

extern "C" int skp_attn_fwd(const float* Q, const float* K, const float* V, float* O, float* stats, int BH, int S,
                            int L, int d, float scale, void* stream) {
  return attn_fwd_launch(Q, contig(S, d), K, contig(L, d), V, contig(L, d), O, contig(S, d), stats, BH, 1, S, L, d,
                         scale, stream);
}

extern "C" int skp_attn_fwd_bshd(const float* Q, long long q_sb, int q_rs, const float* K, long long k_sb, int k_rs,
                                 const float* V, long long v_sb, int v_rs, float* O, long long o_sb, int o_rs,
                                 float* stats, int B, int H, int S, int L, int d, float scale, void* stream) {
  SKP_CHECK_ARG(B > 0 && H > 0 && (long long)B * H <= 65535, "bad B, H");
  return attn_fwd_launch(Q, AttnLay{q_sb, q_rs}, K, AttnLay{k_sb, k_rs}, V, AttnLay{v_sb, v_rs}, O, AttnLay{o_sb, o_rs},
                         stats, B * H, H, S, L, d, scale, stream);
}

// ------------------------------------------------------------------------------------------------
// Fused attention backward over one key block: dS (as skp_attn_dscore), and dV = Pᵀ·dO and
// dK = dSᵀ·Q accumulated in registers across all query rows, so neither P nor dS is read again
// by a GEMM.  Workgroup = 64 keys of one head, 4 waves, looping over 64-row blocks; wave w owns
// rows 16w..16w+15 of each block.  dP = dO·Vᵀ lands in the C layout (lane: rows 4(lane>>4)+r,
// key lane&15), which is the B operand of dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS as it stands, with the
// reduction over rows in the permuted order r = k-step.  The four waves' partial dV / dK are
// summed through LDS at the end (fixed order).
// RC (recompute, skp_attn_bwd_flash): P is not read but rebuilt per row block from Q·Kᵀ on the
// matrix cores (same C layout as dP) and the forward's row stats (m, 1/l), so the forward never
// writes the (B·H, S, L) probabilities.
namespace {

template <int KS, int DB, int WPE, bool RC>   // head dim / 4, 16-wide head-dim blocks, waves per SIMD, recompute P
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void attn_bwd_kv_kernel(
    const float* __restrict__ P, const float* __restrict__ dO, const float* __restrict__ Q, const float* __restrict__ V,
    const float* __restrict__ D, float* __restrict__ dS, float* __restrict__ dV, float* __restrict__ dK, int S, int L,
    float alpha, const float* __restrict__ Kt, const float2* __restrict__ ST, float scale, int H, AttnLay lo, AttnLay lq,
    AttnLay lk, AttnLay lv, AttnLay ldv, AttnLay ldk) {
  constexpr int d = 4 * KS, dp = d + 1, dq = 16 * DB + 1;
  __shared__ float sV[64 * dp];     // this block's keys
  __shared__ float sK[RC ? 64 * dp : 1];
  __shared__ float2 sST[2][RC ? 64 : 1];
  __shared__ float sO[2][64 * dq], sQ[2][64 * dq];   // row blocks of dO and Q, double-buffered (zero-padded to 16·DB)
  __shared__ float sD[2][64];
  const int b = blockIdx.y, k0 = blockIdx.x * 64;   // b = head b·H + h
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float* Vb = lv.at(V, b, H, d);
  const float* dOb = lo.at(dO, b, H, d);
  const float* Qb = lq.at(Q, b, H, d);
  {
    for (int e = t; e < 64 * KS; e += 256) {
      const int key = e / KS, c = 4 * (e - key * KS);
      const bool in = k0 + key < L;   // ragged last block (RC only): keys past L are zero
      const float4 v = in ? *reinterpret_cast<const float4*>(Vb + (size_t)(k0 + key) * lv.rs + c)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      float* p = sV + key * dp + c;
      p[0] = v.x; p[1] = v.y; p[2] = v.z; p[3] = v.w;
      if constexpr (RC) {
        const float4 kk = in ? *reinterpret_cast<const float4*>(lk.at(Kt, b, H, d) + (size_t)(k0 + key) * lk.rs + c)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
        float* pk = sK + key * dp + c;
        pk[0] = kk.x; pk[1] = kk.y; pk[2] = kk.z; pk[3] = kk.w;
      }
    }
    for (int e = t; e < 64 * (dq - d); e += 256) {   // zero pad of the dO / Q tiles (stays zero)
      const int row = e / (dq - d), c = d + (e - row * (dq - d));
      sO[0][row * dq + c] = 0.0f; sO[1][row * dq + c] = 0.0f;
      sQ[0][row * dq + c] = 0.0f; sQ[1][row * dq + c] = 0.0f;
    }
  }
  // the next row block's dO / Q / D / P are fetched into registers at the top of each iteration
  // and dO / Q / D written to the other LDS buffer at its end, so their latency hides under the MFMAs
  constexpr int NPF = (64 * KS + 255) / 256;
  float4 fo[NPF], fq[NPF];
  float fd = 0.0f;
  float2 fst = make_float2(0.0f, 0.0f);
  const int rl = 16 * w + 4 * (lane >> 4);
  auto fetch = [&](int r0) {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int e = t + 256 * j;
      if (e < 64 * KS) {
        const int row = e / KS, c = 4 * (e - row * KS);
        fo[j] = *reinterpret_cast<const float4*>(dOb + (size_t)(r0 + row) * lo.rs + c);
        fq[j] = *reinterpret_cast<const float4*>(Qb + (size_t)(r0 + row) * lq.rs + c);
      }
    }
    if (t < 64) {
      fd = D[(size_t)b * S + r0 + t];
      if constexpr (RC) fst = ST[(size_t)b * S + r0 + t];
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int e = t + 256 * j;
      if (e < 64 * KS) {
        const int row = e / KS, c = 4 * (e - row * KS);
        float* po = sO[buf] + row * dq + c;
        float* pq = sQ[buf] + row * dq + c;
        po[0] = fo[j].x; po[1] = fo[j].y; po[2] = fo[j].z; po[3] = fo[j].w;
        pq[0] = fq[j].x; pq[1] = fq[j].y; pq[2] = fq[j].z; pq[3] = fq[j].w;
      }
    }
    if (t < 64) {
      sD[buf][t] = fd;
      if constexpr (RC) sST[buf][t] = fst;
    }
  };
  // lane's P / dS elements: rows r0 + rl + r, keys k0 + 16bj + (lane&15)
  const float* Pl = P + ((size_t)b * S + rl) * L + k0 + (lane & 15);
  float* dSl = dS + ((size_t)b * S + rl) * L + k0 + (lane & 15);
  f32x4a pc[4];
  if constexpr (!RC) {
#pragma unroll
    for (int bj = 0; bj < 4; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) pc[bj][r] = Pl[(size_t)r * L + 16 * bj];
  }
  fetch(0);
  stash(0);
  f32x4a dv[DB][4], dk[DB][4];
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int bj = 0; bj < 4; ++bj) {
      dv[db][bj] = f32x4a{0.f, 0.f, 0.f, 0.f};
      dk[db][bj] = f32x4a{0.f, 0.f, 0.f, 0.f};
    }
  for (int r0 = 0, buf = 0; r0 < S; r0 += 64, buf ^= 1) {
    __syncthreads();
    const bool more = r0 + 64 < S;
    f32x4a pn[4];
    if (more) {
      fetch(r0 + 64);
      if constexpr (!RC) {
        const float* Pn = Pl + (size_t)(r0 + 64) * L;
#pragma unroll
        for (int bj = 0; bj < 4; ++bj)
#pragma unroll
          for (int r = 0; r < 4; ++r) pn[bj][r] = Pn[(size_t)r * L + 16 * bj];
      }
    }
    const float* tO = sO[buf];
    const float* tQ = sQ[buf];
    // dP = dO·Vᵀ: A = dO[row 16w + (lane&15)][k], B = V[key 16bj + (lane&15)][k], k = 4ks + (lane>>4)
    f32x4a dp4[4];
    {
      const float* oa = tO + (16 * w + (lane & 15)) * dq + (lane >> 4);
      const float* vb = sV + (lane & 15) * dp + (lane >> 4);
#pragma unroll
      for (int bj = 0; bj < 4; ++bj) dp4[bj] = f32x4a{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const float a = oa[4 * ks];
#pragma unroll
        for (int bj = 0; bj < 4; ++bj)
          dp4[bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, vb[16 * bj * dp + 4 * ks], dp4[bj], 0, 0, 0);
      }
    }
    if constexpr (RC) {   // P = exp(scale·Q·Kᵀ − m) / l in the C layout of dP
      f32x4a sc[4];
      const float* qa = tQ + (16 * w + (lane & 15)) * dq + (lane >> 4);
      const float* kb = sK + (lane & 15) * dp + (lane >> 4);
#pragma unroll
      for (int bj = 0; bj < 4; ++bj) sc[bj] = f32x4a{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const float a = qa[4 * ks];
#pragma unroll
        for (int bj = 0; bj < 4; ++bj)
          sc[bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, kb[16 * bj * dp + 4 * ks], sc[bj], 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float2 st = sST[buf][rl + r];
#pragma unroll
        for (int bj = 0; bj < 4; ++bj)
          pc[bj][r] = k0 + 16 * bj + (lane & 15) < L ? __expf(sc[bj][r] * scale - st.x) * st.y : 0.0f;
      }
    }
    f32x4a s4[4];
    float* dSr = dSl + (size_t)r0 * L;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float Dr = sD[buf][rl + r];
#pragma unroll
      for (int bj = 0; bj < 4; ++bj) {
        const float sv = alpha * (pc[bj][r] * (dp4[bj][r] - Dr));
        if (!RC || k0 + 16 * bj + (lane & 15) < L) dSr[(size_t)r * L + 16 * bj] = sv;
        s4[bj][r] = sv;
      }
    }
    // dVᵀ[d][key] += Σ_row dO[row][d] P[row][key]; dKᵀ += Σ_row Q[row][d] dS[row][key];
    // k-step r covers rows 16w + 4(lane>>4) + r
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* orow = tO + (rl + r) * dq + (lane & 15);
      const float* qrow = tQ + (rl + r) * dq + (lane & 15);
#pragma unroll
      for (int db = 0; db < DB; ++db) {
        const float ao = orow[16 * db], aq = qrow[16 * db];
#pragma unroll
        for (int bj = 0; bj < 4; ++bj) {
          dv[db][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(ao, pc[bj][r], dv[db][bj], 0, 0, 0);
          dk[db][bj] = __builtin_amdgcn_mfma_f32_16x16x4f32(aq, s4[bj][r], dk[db][bj], 0, 0, 0);
        }
      }
    }
    if (more) {
      stash(buf ^ 1);
      if constexpr (!RC) {
#pragma unroll
        for (int bj = 0; bj < 4; ++bj) pc[bj] = pn[bj];
      }
    }
  }
  // sum the four waves' partials (LDS, wave order), then lane: dVᵀ[d = 16db + 4(lane>>4) + r'][key
  // 16bj + (lane&15)] → dV[key][d..d+3]
  __syncthreads();
  float* red = sO[0];   // ≥ 64·dq floats; each pass stages one (db, bj) block per wave: 4 × 256 floats
  for (int m = 0; m < 2; ++m) {
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int bj = 0; bj < 4; ++bj) {
        const f32x4a val = m == 0 ? dv[db][bj] : dk[db][bj];
        *reinterpret_cast<float4*>(red + (w * 64 + lane) * 4) = make_float4(val[0], val[1], val[2], val[3]);
        __syncthreads();
        if (w == 0) {
          float4 acc = *reinterpret_cast<const float4*>(red + lane * 4);
#pragma unroll
          for (int ww = 1; ww < 4; ++ww) {
            const float4 x = *reinterpret_cast<const float4*>(red + (ww * 64 + lane) * 4);
            acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
          }
          const int dd = 16 * db + 4 * (lane >> 4);
          const int key = k0 + 16 * bj + (lane & 15);
          if (dd < d && key < L) {
            float* dst = m == 0 ? ldv.at(dV, b, H, d) + (size_t)key * ldv.rs : ldk.at(dK, b, H, d) + (size_t)key * ldk.rs;
            *reinterpret_cast<float4*>(dst + dd) = acc;
          }
        }
        __syncthreads();
      }
  }
}

}  // namespace

extern "C" int skp_attn_bwd_kv(const float* P, const float* dO, const float* Q, const float* V, const float* D,
                               float* dS, float* dV, float* dK, int BH, int S, int L, int d, float alpha,
                               void* stream) {
  SKP_CHECK_ARG(P && dO && Q && V && D && dS && dV && dK, "null pointer");
  SKP_CHECK_ARG(BH > 0 && S > 0 && L > 0, "non-positive shape");
  SKP_CHECK_ARG(S % 64 == 0 && L % 64 == 0, "S and L must be multiples of 64");
  SKP_CHECK_ARG(BH <= 65535, "grid too large");
  SKP_CHECK_ARG(((reinterpret_cast<uintptr_t>(dO) | reinterpret_cast<uintptr_t>(Q) | reinterpret_cast<uintptr_t>(V) |
                  reinterpret_cast<uintptr_t>(dV) | reinterpret_cast<uintptr_t>(dK)) & 15) == 0,
                "tensors must be 16-byte aligned");
  const dim3 grid((unsigned)(L / 64), (unsigned)BH);
  hipStream_t st = as_stream(stream);
  const AttnLay ls = contig(S, d), ll = contig(L, d);
  switch (d) {
#define SKP_BKV(KS_, DB_, W_) \
  hipLaunchKernelGGL((attn_bwd_kv_kernel<KS_, DB_, W_, false>), grid, dim3(256), 0, st, P, dO, Q, V, D, dS, dV, dK, S, L, \
                     alpha, nullptr, nullptr, 0.0f, 1, ls, ls, ll, ll, ll, ll)
    case 40: SKP_BKV(10, 3, 2); break;
    case 64: SKP_BKV(16, 4, 1); break;
    case 80: SKP_BKV(20, 5, 1); break;
#undef SKP_BKV
    default: SKP_CHECK_ARG(false, "head dim must be 40, 64 or 80");
  }
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

namespace {
int attn_bwd_flash_launch(const float* Q, AttnLay lq, const float* K, AttnLay lk, const float* V, AttnLay lv,
                          const float* dO, AttnLay lo, const float* stats, const float* D, float* dS, float* dV,
                          AttnLay ldv, float* dK, AttnLay ldk, int BH, int H, int S, int L, int d, float scale,
                          void* stream) {
  SKP_CHECK_ARG(Q && K && V && dO && stats && D && dS && dV && dK, "null pointer");
  SKP_CHECK_ARG(BH > 0 && H > 0 && BH % H == 0 && S > 0 && L > 0, "non-positive shape");
  SKP_CHECK_ARG(S % 64 == 0, "S must be a multiple of 64");
  SKP_CHECK_ARG(BH <= 65535, "grid too large");
  SKP_CHECK_ARG(((reinterpret_cast<uintptr_t>(dO) | reinterpret_cast<uintptr_t>(Q) | reinterpret_cast<uintptr_t>(K) |
                  reinterpret_cast<uintptr_t>(V) | reinterpret_cast<uintptr_t>(dV) | reinterpret_cast<uintptr_t>(dK)) &
                 15) == 0 && (reinterpret_cast<uintptr_t>(stats) & 7) == 0,
                "tensors must be 16-byte aligned (stats 8-byte)");
  SKP_CHECK_ARG(((lq.rs | lk.rs | lv.rs | lo.rs | ldv.rs | ldk.rs | lq.sb | lk.sb | lv.sb | lo.sb | ldv.sb | ldk.sb) & 3) == 0,
                "strides must be multiples of 4");
  const dim3 grid((unsigned)((L + 63) / 64), (unsigned)BH);
  hipStream_t st = as_stream(stream);
  const float2* ST = reinterpret_cast<const float2*>(stats);
  switch (d) {
#define SKP_BFL(KS_, DB_, W_) \
  hipLaunchKernelGGL((attn_bwd_kv_kernel<KS_, DB_, W_, true>), grid, dim3(256), 0, st, nullptr, dO, Q, V, D, dS, dV, dK, \
                     S, L, scale, K, ST, scale, H, lo, lq, lk, lv, ldv, ldk)
    case 40: SKP_BFL(10, 3, 2); break;
    case 64: SKP_BFL(16, 4, 1); break;
    case 80: SKP_BFL(20, 5, 1); break;
#undef SKP_BFL
    default: SKP_CHECK_ARG(false, "head dim must be 40, 64 or 80");
  }
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
}  // namespace

extern "C" int skp_attn_bwd_flash(const float* Q, const float* K, const float* V, const float* dO, const float* stats,
                                  const float* D, float* dS, float* dV, float* dK, int BH, int S, int L, int d, float scale,
                                  void* stream) {
  const AttnLay ls = contig(S, d), ll = contig(L, d);
  return attn_bwd_flash_launch(Q, ls, K, ll, V, ll, dO, ls, stats, D, dS, dV, ll, dK, ll, BH, 1, S, L, d, scale, stream);
}

extern "C" int skp_attn_bwd_flash_bshd(const float* Q, long long q_sb, int q_rs, const float* K, long long k_sb,
                                       int k_rs, const float* V, long long v_sb, int v_rs, const float* dO,
                                       long long o_sb, int o_rs, const float* stats, const float* D, float* dS,
                                       float* dV, long long dv_sb, int dv_rs, float* dK, long long dk_sb, int dk_rs,
                                       int B, int H, int S, int L, int d, float scale, void* stream) {
  SKP_CHECK_ARG(B > 0 && H > 0 && (long long)B * H <= 65535, "bad B, H");
  return attn_bwd_flash_launch(Q, AttnLay{q_sb, q_rs}, K, AttnLay{k_sb, k_rs}, V, AttnLay{v_sb, v_rs}, dO,
                               AttnLay{o_sb, o_rs}, stats, D, dS, dV, AttnLay{dv_sb, dv_rs}, dK, AttnLay{dk_sb, dk_rs},
                               B * H, H, S, L, d, scale, stream);
}
