// Strided batched fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32,
// k-ordered fma chain) for the capture logits z = q kᵀ·scale (ptp_utils.py:493/534) and
// their gradients dq = dz k·scale, dk = dzᵀ q·scale.
//
// Shapes on the hot path are small (batch·heads = 8, M = s² ≤ 1024, N = tokens ≤ 1024,
// K = head dim 40..160), so each 256-thread workgroup computes one 64×64 C tile as 2×2
// waves of 32×32 and stages the K-panel of A and B through LDS in 16-deep slices.
#include "skp_common.h"

using namespace skp;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BN = 64, BK = 16;

__global__ __launch_bounds__(256) void bgemm_kernel(const float* __restrict__ A, long long sAb, long long sAm,
                                                    long long sAk, const float* __restrict__ B, long long sBb,
                                                    long long sBk, long long sBn, float* __restrict__ C, long long sCb,
                                                    long long sCm, long long sCn, int M, int N, int K, float alpha,
                                                    int accumulate) {
  __shared__ float As[BK][BM + 1];
  __shared__ float Bs[BK][BN + 1];
  const int bz = blockIdx.z;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const float* Ab = A + bz * sAb;
  const float* Bb = B + bz * sBb;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  for (int k0 = 0; k0 < K; k0 += BK) {
    // stage A[m0:m0+64, k0:k0+16] and B[k0:k0+16, n0:n0+64]; pick the thread order that
    // walks the unit-stride dimension across lanes.
    for (int e = t; e < BM * BK; e += 256) {
      int mm, kk;
      if (sAk == 1) { mm = e / BK; kk = e % BK; } else { kk = e / BM; mm = e % BM; }
      const int m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < M && k < K) ? Ab[m * sAm + k * sAk] : 0.0f;
    }
    for (int e = t; e < BN * BK; e += 256) {
      int nn, kk;
      if (sBk == 1) { nn = e / BK; kk = e % BK; } else { kk = e / BN; nn = e % BN; }
      const int n = n0 + nn, k = k0 + kk;
      Bs[kk][nn] = (n < N && k < K) ? Bb[k * sBk + n * sBn] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = As[kk + (lane >> 5)][wm + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wn + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
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

}  // namespace

extern "C" int skp_bgemm_f32(const float* A, long long sAb, long long sAm, long long sAk, const float* B,
                             long long sBb, long long sBk, long long sBn, float* C, long long sCb, long long sCm,
                             long long sCn, int batch, int M, int N, int K, float alpha, int accumulate,
                             void* stream) {
  SKP_CHECK_ARG(A && B && C, "null pointer");
  SKP_CHECK_ARG(batch > 0 && M > 0 && N > 0 && K > 0, "non-positive shape");
  SKP_CHECK_ARG(batch <= 65535, "batch > 65535");
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch);
  hipLaunchKernelGGL(bgemm_kernel, grid, dim3(256), 0, as_stream(stream), A, sAb, sAm, sAk, B, sBb, sBk, sBn, C, sCb,
                     sCm, sCn, M, N, K, alpha, accumulate);
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}
