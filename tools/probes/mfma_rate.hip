// MFMA issue-rate probe (dev tool): cycles per f32 MFMA on gfx950 for dependent / independent
// accumulator chains and 1..4 waves per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CHAINS, bool BIG>
__global__ __launch_bounds__(256) void probe(float* out, int iters, long long* cyc) {
  float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
  f32x16 acc16[CHAINS];
  f32x4 acc4[CHAINS];
  for (int c = 0; c < CHAINS; ++c) { acc16[c] = (f32x16)0.0f; acc4[c] = (f32x4)0.0f; }
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if (BIG) acc16[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc16[c], 0, 0, 0);
      else acc4[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc4[c], 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = 0;
  for (int c = 0; c < CHAINS; ++c) s += BIG ? acc16[c][0] + acc16[c][15] : acc4[c][0] + acc4[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int CHAINS, bool BIG>
void run(int waves_per_simd) {
  const int iters = 4096;
  float* out;
  long long* cyc;
  hipMalloc(&out, 1024 * 256 * 4 * sizeof(float));
  hipMalloc(&cyc, sizeof(long long));
  const int blocks = 256 * waves_per_simd;   // 256 threads = 4 waves = one per SIMD per block
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<CHAINS, BIG><<<blocks, 256>>>(out, iters, cyc);
  hipEventRecord(e0);
  probe<CHAINS, BIG><<<blocks, 256>>>(out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long c;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  const double flops = (double)blocks * 4 * iters * CHAINS * (BIG ? 32.0 * 32 * 2 * 2 : 16.0 * 16 * 4 * 2);
  printf("%s chains=%d waves/SIMD=%d: %.1f TF/s, %.1f clock64 ticks per MFMA per wave\n",
         BIG ? "32x32x2" : "16x16x4", CHAINS, waves_per_simd, flops / (ms * 1e-3) / 1e12,
         (double)c / (iters * CHAINS));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w : {1, 2, 4}) {
    run<1, true>(w);
    run<4, true>(w);
    run<1, false>(w);
    run<4, false>(w);
  }
  return 0;
}
