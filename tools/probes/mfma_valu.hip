// Probe (dev tool): does VALU work overlap an f32 MFMA on gfx950?  Each iteration issues one MFMA
// (16x16x4 f32 or 32x32x2 f32, dependent chain) and NV independent VALU ops (v_fma_f32 or
// v_pk_fma_f32) from the same wave; reports clock64 ticks per iteration for 1 and 2 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NV, bool PK, bool BIG>
__global__ __launch_bounds__(256) void probe(float* out, int iters, long long* cyc) {
  const float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
  f32x4 acc = (f32x4)0.0f;
  f32x16 acc16 = (f32x16)0.0f;
  float v[8];
  f32x2 w[8];
  for (int i = 0; i < 8; ++i) { v[i] = i * 0.1f + a; w[i] = (f32x2){v[i], b}; }
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (BIG) acc16 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc16, 0, 0, 0);
    else acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      if (PK) w[j & 7] = __builtin_elementwise_fma(w[j & 7], (f32x2){1.0001f, 0.9999f}, (f32x2){1e-7f, 2e-7f});
      else v[j & 7] = __builtin_fmaf(v[j & 7], 1.0001f, 1e-7f);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  const long long t1 = clock64();
  float s = BIG ? acc16[0] : acc[0];
  for (int i = 0; i < 8; ++i) s += v[i] + w[i][0] + w[i][1];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int NV, bool PK, bool BIG>
void run(int wps) {
  const int iters = 20000, blocks = 256 * wps;
  float* out;
  long long* cyc;
  (void)hipMalloc(&out, blocks * 256 * sizeof(float));
  (void)hipMalloc(&cyc, sizeof(long long));
  probe<NV, PK, BIG><<<blocks, 256>>>(out, iters, cyc);
  (void)hipDeviceSynchronize();
  long long c;
  (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%s + %2d %s, %d wave/SIMD: %.1f ticks/iter\n", BIG ? "32x32x2" : "16x16x4", NV, PK ? "v_pk_fma" : "v_fma   ", wps,
         (double)c / iters);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  for (int w : {1, 2}) {
    run<0, false, false>(w); run<2, false, false>(w); run<4, false, false>(w); run<6, false, false>(w);
    run<8, false, false>(w); run<12, false, false>(w); run<16, false, false>(w);
    run<2, true, false>(w); run<4, true, false>(w); run<8, true, false>(w);
    run<0, false, true>(w); run<8, false, true>(w); run<16, false, true>(w); run<8, true, true>(w);
  }
  return 0;
}
