// Strided batched fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32
// products, fp32 accumulation) for the capture logits z = q kᵀ·scale (ptp_utils.py:493/534) and
// their gradients dq = dz k·scale, dk = dzᵀ q·scale.
//
// Shapes on the hot path are small (batch·heads = 64, M = s² ≤ 1024, N = tokens ≤ 1024, K = head
// dim 40..160 or tokens/pixels for the gradients), so a 64×64 tile owns only 5 panels of 32 k
// and a one-tile-per-workgroup grid exposes every tile's first loads and its epilogue (r01: 28–36%
// of the 157 TF/s f32 MFMA peak).  Here the grid is persistent (4 workgroups per CU, XCD-aware): each
// workgroup walks its tiles as one flat sequence of (tile, k-panel) steps, the next step's global
// loads (possibly the next tile's first panel) fly in registers during this step's MFMAs, and a
// finished tile's epilogue stores overlap the next step, so the pipeline drains once per workgroup.
//
// One 256-thread workgroup computes a 64×64 C tile as 2×2 waves of 32×32.  Operand layouts in
// LDS follow the global unit stride, with no transpose on the way in:
//   k unit stride   -> [mn][k] rows of 32 k (+4 pad): one ds_read_b128 gives a lane 4 k values;
//   m/n unit stride -> [k][mn] rows of 64 (+4 pad): one ds_read_b32 per k (row-contiguous lanes).
// MFMA j (0..3) of k-group g takes k = 8g + j from lanes 0-31 and k = 8g + 4 + j from lanes
// 32-63, for both operands, so each k-group is 4 MFMAs fed by one b128 read (k-order within the
// fp32 sum differs from a plain chain, as any blocked GEMM's does).
#include <algorithm>
#include <cstdlib>

#include "skp_common.h"

using namespace skp;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDK = BK + 4;       // [mn][k] row stride (floats): 16-B aligned, b128 reads spread over banks
constexpr int kOcc = 4;           // workgroups per CU for 64×64 tiles (LDS 36.9 KB each)

// v where m = −1, +0.0 where m = 0: integer masking of an unconditional load (a select lets the
// compiler turn the load into an exec-masked one after zeroing its destination: a vmcnt(0))
__device__ __forceinline__ float4 keep_or_zero(float4 v, int m) {
  return make_float4(__int_as_float(__float_as_int(v.x) & m), __int_as_float(__float_as_int(v.y) & m),
                     __int_as_float(__float_as_int(v.z) & m), __int_as_float(__float_as_int(v.w) & m));
}

// Operand panel loader for a BMN-wide tile edge: BK·BMN/4 float4 slots over NT threads.
// MODE 0: unit stride along k; 1: unit stride along m/n; 2: generic (scalar loads).
// Branch-free: out-of-range quads load a clamped in-range address and are zeroed when the panel
// goes to LDS (MODE 0 needs K % 4 == 0 and MODE 1 MN % 4 == 0, so a quad is all in or all out;
// the host sends other operands down MODE 2).  Straight-line loads with no instruction touching
// their registers before the LDS store keep the waitcnt counting exact, so the prefetch really
// stays in flight across the MFMAs.
template <int MODE, int BMN, int NT>
struct Loader {
  static constexpr int NS = BMN * BK / 4 / NT;   // float4 slots per thread
  static constexpr int LDM = BMN + 4;   // [k][mn] row stride
  static constexpr int QK = BK / 4;     // MODE 0: float4 slots along k per m/n
  static constexpr int QM = BMN / 4;    // MODE 1/2: float4 slots along m/n per k
  float4 r[NS];
  int keep[NS];
  int keepu[NS][4];
  __device__ __forceinline__ void load(const float* __restrict__ P, long long sk, long long smn, int k0, int mn0, int K,
                                       int MN) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int e = threadIdx.x + i * NT;
      if (MODE == 0) {
        const int mn = mn0 + e / QK, k = k0 + 4 * (e % QK);
        r[i] = *reinterpret_cast<const float4*>(P + min(mn, MN - 1) * smn + min(k, K - 4));
        keep[i] = -(int)(mn < MN && k < K);
      } else if (MODE == 1) {
        const int k = k0 + e / QM, mn = mn0 + 4 * (e % QM);
        r[i] = *reinterpret_cast<const float4*>(P + min(k, K - 1) * sk + min(mn, MN - 4));
        keep[i] = -(int)(k < K && mn < MN);
      } else {
        const int k = k0 + e / QM, mn = mn0 + 4 * (e % QM);
        const int kc = min(k, K - 1);
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          keepu[i][u] = -(int)(k < K && mn + u < MN);
          v[u] = P[kc * sk + min(mn + u, MN - 1) * smn];
        }
        r[i] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ S) const {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int e = threadIdx.x + i * NT;
      float4 v;
      if (MODE < 2) {
        v = keep_or_zero(r[i], keep[i]);
      } else {
        v = make_float4(__int_as_float(__float_as_int(r[i].x) & keepu[i][0]),
                        __int_as_float(__float_as_int(r[i].y) & keepu[i][1]),
                        __int_as_float(__float_as_int(r[i].z) & keepu[i][2]),
                        __int_as_float(__float_as_int(r[i].w) & keepu[i][3]));
      }
      if (MODE == 0) *reinterpret_cast<float4*>(S + (e / QK) * LDK + 4 * (e % QK)) = v;
      else *reinterpret_cast<float4*>(S + (e / QM) * LDM + 4 * (e % QM)) = v;
    }
  }
  // this lane's 4 operand values of k-group g (k = 8g + 4h + j, j = 0..3) at m/n offset mn
  __device__ __forceinline__ static float4 frag(const float* __restrict__ S, int g, int h, int mn) {
    if (MODE == 0) return *reinterpret_cast<const float4*>(S + mn * LDK + 8 * g + 4 * h);
    const float* p = S + (8 * g + 4 * h) * LDM + mn;
    return make_float4(p[0], p[LDM], p[2 * LDM], p[3 * LDM]);
  }
  static constexpr int kBuf = (BMN * LDK > BK * LDM) ? BMN * LDK : BK * LDM;   // floats per buffer
};

// BM×BN tile per workgroup as WM×WN waves of (BM/WM)×(BN/WN), each a grid of MI×NI 32×32 MFMA blocks
// Batch index bz = o·hb + i (o < batch / hb): operand X's base is X + o·sXo + i·sXb, so a (B, S, H·d)
// projection is a batch of B·H (S, d) heads in place (sXo = S·H·d, sXb = d, rows H·d apart) and an
// operand shared by the B images is sXo = 0 — no head-permute or batch-expand copies (hb = batch,
// sXo = 0: the plain one-stride batch).
template <int MA, int MB, bool ACC, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * WAVE) void bgemm_kernel(const float* __restrict__ A, long long sAb, long long sAm,
                                                         long long sAk, const float* __restrict__ B, long long sBb,
                                                         long long sBk, long long sBn, float* __restrict__ C,
                                                         long long sCb, long long sCm, long long sCn, int M, int N,
                                                         int K, float alpha, int tiles_m, int tiles_n, int tiles,
                                                         int hb, long long sAo, long long sBo, long long sCo) {
  constexpr int NT = WM * WN * WAVE;
  using LA = Loader<MA, BM, NT>;
  using LB = Loader<MB, BN, NT>;
  constexpr int MI = BM / WM / 32, NI = BN / WN / 32;
  __shared__ __attribute__((aligned(16))) float As[2][LA::kBuf];
  __shared__ __attribute__((aligned(16))) float Bs[2][LB::kBuf];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid / WN) * (BM / WM), wn = (wid % WN) * (BN / WN);
  const int h = lane >> 5, r = lane & 31;
  const int npanel = (K + BK - 1) / BK;
  // XCD-aware tile order: workgroup b runs on XCD b % 8, and XCD x owns the contiguous tile range
  // [x·per, x·per + per) (batch-major, tn fastest), walked by its gridDim/8 workgroups — each
  // batch's q and k rows are then fetched into one XCD's L2 and reused there by all its tiles
  const int G = (int)gridDim.x >> 3;   // workgroups per XCD (the grid is a multiple of 8)
  const int per = (tiles + 7) / 8;
  const int t0 = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
  const int span = min(tiles, ((int)blockIdx.x & 7) * per + per) - t0;
  const int mine = span > 0 ? (span - 1) / G + 1 : 0;
  if (mine == 0) return;
  LA la;
  LB lb;
  // tile t = (bz·tiles_m + tm)·tiles_n + tn; the loads run one step ahead of the MFMAs, so the
  // loader keeps its own (tile, panel) cursor, advanced without divisions (one decode per tile).
  // (Two steps ahead in two register sets measured slower: 37.1 vs 36.1 us at the bench's q kᵀ.)
  struct Cursor {
    int ti, p, m0, n0;
    const float *a, *b;
  };
  auto decode = [&](int ti, Cursor& c) {
    const int t = t0 + ti * G;
    const int tn = t % tiles_n, tm = (t / tiles_n) % tiles_m, bz = t / (tiles_n * tiles_m);
    c.ti = ti;
    c.p = 0;
    c.m0 = tm * BM;
    c.n0 = tn * BN;
    const int bo = bz / hb, bi = bz - bo * hb;
    c.a = A + bo * sAo + bi * sAb;
    c.b = B + bo * sBo + bi * sBb;
  };
  Cursor ld;
  decode(0, ld);
  auto issue = [&]() {
    la.load(ld.a, sAk, sAm, ld.p * BK, ld.m0, K, M);   // A viewed as [k][m]
    lb.load(ld.b, sBk, sBn, ld.p * BK, ld.n0, K, N);   // B viewed as [k][n]
  };
  auto advance = [&]() {   // to the next step (the last step stays put: it re-loads itself)
    if (ld.p + 1 < npanel) ++ld.p;
    else if (ld.ti + 1 < mine) decode(ld.ti + 1, ld);
  };
  issue();
  advance();
  la.store(As[0]);
  lb.store(Bs[0]);
  __syncthreads();
  int s = 0;
  for (int ti = 0; ti < mine; ++ti) {
    f32x16 acc[MI][NI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[mi][ni][i] = 0.0f;
    for (int p = 0; p < npanel; ++p, ++s) {
      const int cur = s & 1;
      // next step's loads (maybe the next tile's first panel) fly during the MFMAs; the last step
      // re-loads itself into the idle buffer, so the loads need no branch (and no phi copies)
      issue();
      advance();
      __builtin_amdgcn_sched_barrier(0);   // keep the loads ahead of the MFMAs (the scheduler sinks them)
      const float* as = As[cur];
      const float* bs = Bs[cur];
#pragma unroll
      for (int g = 0; g < BK / 8; ++g) {
        float4 a[MI], b[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) a[mi] = LA::frag(as, g, h, wm + 32 * mi + r);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) b[ni] = LB::frag(bs, g, h, wn + 32 * ni + r);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mi].x, b[ni].x, acc[mi][ni], 0, 0, 0);
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mi].y, b[ni].y, acc[mi][ni], 0, 0, 0);
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mi].z, b[ni].z, acc[mi][ni], 0, 0, 0);
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mi].w, b[ni].w, acc[mi][ni], 0, 0, 0);
          }
      }
      la.store(As[cur ^ 1]);
      lb.store(Bs[cur ^ 1]);
      // tile done: its stores go out AFTER the prefetched panel reached LDS (vmcnt counts loads and
      // stores in issue order, so stores issued first would add their acks to that wait)
      if (p == npanel - 1) {
        const int t = t0 + ti * G;
        const int tn = t % tiles_n, tm = (t / tiles_n) % tiles_m, bz = t / (tiles_n * tiles_m);
        const int bo = bz / hb, bi = bz - bo * hb;
        float* Cb = C + bo * sCo + bi * sCb;
        // materialise the tile's row/column bases here: otherwise LICM hoists all MI·NI·16 store
        // addresses out of the panel loop and keeps them live across the MFMAs (register blow-up)
        int rb = tm * BM + wm + 4 * h, cb = tn * BN + wn + r;
        asm volatile("" : "+v"(rb), "+v"(cb));
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            const int col = cb + 32 * ni;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int row = rb + 32 * mi + (i & 3) + 8 * (i >> 2);
              if (row < M && col < N) {
                float* q = Cb + row * sCm + col * sCn;
                const float v = alpha * acc[mi][ni][i];
                if (ACC) *q += v;   // read-modify-write only in the accumulate instantiation
                else *q = v;
              }
            }
          }
      }
      __syncthreads();
    }
  }
}

int mode_of(const void* P, long long sk, long long smn, int k, int mn) {
  const bool al = (reinterpret_cast<uintptr_t>(P) & 15) == 0;
  if (sk == 1 && al && smn % 4 == 0 && k % 4 == 0) return 0;
  if (smn == 1 && al && sk % 4 == 0 && mn % 4 == 0) return 1;
  return 2;
}

}  // namespace

extern "C" int skp_bgemm_f32_2b(const float* A, long long sAo, long long sAb, long long sAm, long long sAk,
                                const float* B, long long sBo, long long sBb, long long sBk, long long sBn, float* C,
                                long long sCo, long long sCb, long long sCm, long long sCn, int batch, int hb, int M,
                                int N, int K, float alpha, int accumulate, void* stream) {
  SKP_CHECK_ARG(A && B && C, "null pointer");
  SKP_CHECK_ARG(batch > 0 && M > 0 && N > 0 && K > 0, "non-positive shape");
  SKP_CHECK_ARG(batch <= 65535, "batch > 65535");
  SKP_CHECK_ARG(hb > 0 && batch % hb == 0, "hb must divide batch");
  const int ma = mode_of(A, sAk, sAm, K, M), mb = mode_of(B, sBk, sBn, K, N);
  // batch strides must keep each batch's base aligned for the vector paths
  const int fa = (ma < 2 && (sAb % 4 != 0 || sAo % 4 != 0)) ? 2 : ma;
  const int fb = (mb < 2 && (sBb % 4 != 0 || sBo % 4 != 0)) ? 2 : mb;
  // tile edge per dimension: 128 (twice the flops per loaded byte) unless its padding wastes more
  // than 64's; 128×128 runs 2 workgroups per CU (73.7 KB LDS), the others 4 (or 3)
  auto pick = [](int n) {
    const int w64 = (n + 63) / 64 * 64, w128 = (n + 127) / 128 * 128;
    return (w128 - n) <= (w64 - n) + n / 16 ? 128 : 64;
  };
  int bm = pick(M), bn = pick(N);
  if (fa == 2 || fb == 2) bm = bn = 64;
  const long long tiles128 = (long long)batch * ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  if (tiles128 < 512) bm = bn = 64;   // too few tiles to fill 256 CUs twice: keep the small tile
  const int tiles_m = (M + bm - 1) / bm, tiles_n = (N + bn - 1) / bn;
  const long long tiles = (long long)batch * tiles_m * tiles_n;
  SKP_CHECK_ARG(tiles < (1LL << 31), "too many tiles");
  // workgroups per CU (occupancy at 1, 2 or 3 per CU measured the same on q·kᵀ)
  const int occ = (bm == 128 && bn == 128) ? 2 : (bm == 128 || bn == 128) ? 3 : kOcc;
  const int grid = (int)std::min<long long>(8 * ((tiles + 7) / 8), 256LL * occ) & ~7;
  hipStream_t st = as_stream(stream);
#define SKP_BG3(X, Y, TM, TN, WM, WN)                                                                           \
  if (accumulate)                                                                                               \
    hipLaunchKernelGGL((bgemm_kernel<X, Y, true, TM, TN, WM, WN>), dim3(grid), dim3(WM * WN * WAVE), 0, st, A,  \
                       sAb, sAm, sAk, B, sBb, sBk, sBn, C, sCb, sCm, sCn, M, N, K, alpha, tiles_m, tiles_n,     \
                       (int)tiles, hb, sAo, sBo, sCo);                                                          \
  else                                                                                                          \
    hipLaunchKernelGGL((bgemm_kernel<X, Y, false, TM, TN, WM, WN>), dim3(grid), dim3(WM * WN * WAVE), 0, st, A, \
                       sAb, sAm, sAk, B, sBb, sBk, sBn, C, sCb, sCm, sCn, M, N, K, alpha, tiles_m, tiles_n,     \
                       (int)tiles, hb, sAo, sBo, sCo)
  // 128-edge tiles run 8 waves (4 per SIMD at two workgroups per CU)
#define SKP_BG(X, Y)                                                         \
  if (X == 2 || Y == 2 || (bm == 64 && bn == 64)) {                          \
    SKP_BG3(X, Y, 64, 64, 2, 2);                                             \
  } else if (bm == 128 && bn == 128) {                                       \
    SKP_BG3((X < 2 ? X : 0), (Y < 2 ? Y : 0), 128, 128, 4, 2);               \
  } else if (bm == 128) {                                                    \
    SKP_BG3((X < 2 ? X : 0), (Y < 2 ? Y : 0), 128, 64, 2, 2);                \
  } else {                                                                   \
    SKP_BG3((X < 2 ? X : 0), (Y < 2 ? Y : 0), 64, 128, 2, 2);                \
  }
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
#undef SKP_BG3
  SKP_LAUNCH_CHECK();
  return SKP_OK;
}

extern "C" int skp_bgemm_f32(const float* A, long long sAb, long long sAm, long long sAk, const float* B,
                             long long sBb, long long sBk, long long sBn, float* C, long long sCb, long long sCm,
                             long long sCn, int batch, int M, int N, int K, float alpha, int accumulate,
                             void* stream) {
  return skp_bgemm_f32_2b(A, 0, sAb, sAm, sAk, B, 0, sBb, sBk, sBn, C, 0, sCb, sCm, sCn, batch, batch, M, N, K, alpha,
                          accumulate, stream);
}
