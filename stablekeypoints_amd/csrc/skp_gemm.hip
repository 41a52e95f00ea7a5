// Strided batched fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32,
// k-ordered fma chain) for the capture logits z = q kᵀ·scale (ptp_utils.py:493/534) and
// their gradients dq = dz k·scale, dk = dzᵀ q·scale.
//
// Shapes on the hot path are small (batch·heads = 8..16, M = s² ≤ 1024, N = tokens ≤ 1024,
// K = head dim 40..160 or tokens/pixels for the gradients).  One 256-thread workgroup computes
// a 64×64 C tile as 2×2 waves of 32×32.  K is walked in 32-deep panels: the next panel's global
// loads are issued into registers before the current panel's 16 MFMAs per wave, then written
// to the other LDS buffer (one barrier per panel).  Loads are 16-B vectors along whichever of
// the operand's two dimensions is unit-stride (k, or m/n), so all four operand layouts of the
// forward and backward products read coalesced.
#include "skp_common.h"

using namespace skp;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BN = 64, BK = 32;
constexpr int kThreads = 256;
constexpr int LDA = BM + 4;   // padded LDS rows (floats): keeps float4 stores aligned, spreads banks
constexpr int LDB = BN + 4;

// Operand tile loader: the tile is [BK rows (k)] × [64 cols (m or n)] in LDS (k-major).
// MODE 0: unit stride along k (float4 over k); 1: unit stride along m/n (float4 over m/n);
// 2: generic (scalar).  Each thread loads 8 floats (2 float4) per panel.
template <int MODE>
struct Loader {
  float4 r[2];
  __device__ __forceinline__ void load(const float* __restrict__ P, long long sk, long long smn, int k0, int mn0, int K,
                                       int MN) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = threadIdx.x + i * kThreads;   // 512 float4 slots = 32 × 64 floats
      if (MODE == 0) {          // 8 float4 along k per column: col = e / 8, kq = e % 8
        const int col = e >> 3, kq = e & 7;
        const int mn = mn0 + col, k = k0 + 4 * kq;
        if (mn < MN && k + 3 < K) {
          r[i] = *reinterpret_cast<const float4*>(P + mn * smn + k);
        } else {
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = (mn < MN && k + u < K) ? P[mn * smn + (k + u)] : 0.0f;
          r[i] = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else if (MODE == 1) {   // 16 float4 along m/n per k row: kk = e / 16, cq = e % 16
        const int kk = e >> 4, cq = e & 15;
        const int k = k0 + kk, mn = mn0 + 4 * cq;
        if (k < K && mn + 3 < MN) {
          r[i] = *reinterpret_cast<const float4*>(P + k * sk + mn);
        } else {
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = (k < K && mn + u < MN) ? P[k * sk + (mn + u)] : 0.0f;
          r[i] = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {                  // scalar: same slot geometry as MODE 1
        const int kk = e >> 4, cq = e & 15;
        const int k = k0 + kk, mn = mn0 + 4 * cq;
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = (k < K && mn + u < MN) ? P[k * sk + (mn + u) * smn] : 0.0f;
        r[i] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ S, int ld) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = threadIdx.x + i * kThreads;
      if (MODE == 0) {
        const int col = e >> 3, kq = e & 7;
        S[(4 * kq + 0) * ld + col] = r[i].x;
        S[(4 * kq + 1) * ld + col] = r[i].y;
        S[(4 * kq + 2) * ld + col] = r[i].z;
        S[(4 * kq + 3) * ld + col] = r[i].w;
      } else {
        const int kk = e >> 4, cq = e & 15;
        *reinterpret_cast<float4*>(S + kk * ld + 4 * cq) = r[i];
      }
    }
  }
};

template <int MA, int MB>
__global__ __launch_bounds__(kThreads) void bgemm_kernel(const float* __restrict__ A, long long sAb, long long sAm,
                                                         long long sAk, const float* __restrict__ B, long long sBb,
                                                         long long sBk, long long sBn, float* __restrict__ C,
                                                         long long sCb, long long sCm, long long sCn, int M, int N,
                                                         int K, float alpha, int accumulate) {
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB];
  const int bz = blockIdx.z;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const float* Ab = A + bz * sAb;
  const float* Bb = B + bz * sBb;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  Loader<MA> la;
  Loader<MB> lb;
  // A viewed as [k][m]: (sk = sAk, smn = sAm); B as [k][n]: (sk = sBk, smn = sBn)
  la.load(Ab, sAk, sAm, 0, m0, K, M);
  lb.load(Bb, sBk, sBn, 0, n0, K, N);
  la.store(As[0], LDA);
  lb.store(Bs[0], LDB);
  __syncthreads();
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  const int npanel = (K + BK - 1) / BK;
  for (int p = 0; p < npanel; ++p) {
    const int cur = p & 1;
    const bool more = p + 1 < npanel;
    if (more) {   // next panel's loads fly during this panel's MFMAs
      la.load(Ab, sAk, sAm, (p + 1) * BK, m0, K, M);
      lb.load(Bb, sBk, sBn, (p + 1) * BK, n0, K, N);
    }
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = as[(kk + (lane >> 5)) * LDA + wm + (lane & 31)];
      const float b = bs[(kk + (lane >> 5)) * LDB + wn + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    if (more) {
      la.store(As[cur ^ 1], LDA);
      lb.store(Bs[cur ^ 1], LDB);
    }
    __syncthreads();
  }
  float* Cb = C + bz * sCb;
  const int col = n0 + wn + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < M && col < N) {
      float* p = Cb + row * sCm + col * sCn;
      const float v = alpha * acc[r];
      *p = accumulate ? (*p + v) : v;
    }
  }
}

int mode_of(const void* P, long long sk, long long smn) {
  const bool al = (reinterpret_cast<uintptr_t>(P) & 15) == 0;
  if (sk == 1 && al && smn % 4 == 0) return 0;
  if (smn == 1 && al && sk % 4 == 0) return 1;
  return 2;
}

}  // namespace

extern "C" int skp_bgemm_f32(const float* A, long long sAb, long long sAm, long long sAk, const float* B,
                             long long sBb, long long sBk, long long sBn, float* C, long long sCb, long long sCm,
                             long long sCn, int batch, int M, int N, int K, float alpha, int accumulate,
                             void* stream) {
  SKP_CHECK_ARG(A && B && C, "null pointer");
  SKP_CHECK_ARG(batch > 0 && M > 0 && N > 0 && K > 0, "non-positive shape");
  SKP_CHECK_ARG(batch <= 65535, "batch > 65535");
  const int ma = mode_of(A, sAk, sAm), mb = mode_of(B, sBk, sBn);
  // batch strides must keep each batch's base aligned for the vector paths
  const int fa = (ma < 2 && sAb % 4 != 0) ? 2 : ma;
  const int fb = (mb < 2 && sBb % 4 != 0) ? 2 : mb;
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch);
  hipStream_t st = as_stream(stream);
#define SKP_BG(X, Y)                                                                                          \
  hipLaunchKernelGGL((bgemm_kernel<X, Y>), grid, dim3(kThreads), 0, st, A, sAb, sAm, sAk, B, sBb, sBk, sBn, C, \
                     sCb, sCm, sCn, M, N, K, alpha, accumulate)
  switch (fa * 3 + fb) {
    case 0: SKP_BG(0, 0); break;
    case 1: SKP_BG(0, 1); break;
    case 2: SKP_BG(0, 2); break;
    case 3: SKP_BG(1, 0); break;
    case 4: SKP_BG(1, 1); break;
    case 5: SKP_BG(1, 2); break;
    case 6: SKP_BG(2, 0); break;
    case 7: SKP_BG(2, 1); break;
    default: SKP_BG(2, 2); break;
  }
#undef SKP_BG
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
