// Probe (dev tool): f32 MFMA rate inside the bgemm step structure — per step each wave reads its
// fragments from LDS (ds_read_b128), runs 16 v_mfma_f32_32x32x2_f32, writes 4 float4 to the other
// LDS buffer and meets a workgroup barrier — without global memory.  Occupancy 1..4 workgroups/CU.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int LDK = 36, OPB = 64 * LDK;

template <int MODE>   // 0: barrier + LDS write per step; 1: LDS reads only; 2: MFMA only
__global__ __launch_bounds__(256) void probe(float* out, int steps) {
  __shared__ __attribute__((aligned(16))) float As[2][OPB];
  __shared__ __attribute__((aligned(16))) float Bs[2][OPB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32, h = lane >> 5, r = lane & 31;
  for (int i = threadIdx.x; i < 2 * OPB; i += 256) { (&As[0][0])[i] = i * 1e-4f; (&Bs[0][0])[i] = 1 - i * 1e-5f; }
  __syncthreads();
  f32x16 acc = (f32x16)0.0f;
  float4 keep = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < steps; ++s) {
    const int cur = MODE == 0 ? (s & 1) : 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float4 a, b;
      if (MODE < 2) {
        a = *reinterpret_cast<const float4*>(&As[cur][(wm + r) * LDK + 8 * g + 4 * h]);
        b = *reinterpret_cast<const float4*>(&Bs[cur][(wn + r) * LDK + 8 * g + 4 * h]);
      } else {
        a = make_float4(g, h, r, s);
        b = a;
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
    }
    if (MODE == 0) {
      keep.x += acc[0];
      const int e = threadIdx.x;
      *reinterpret_cast<float4*>(&As[cur ^ 1][(e >> 3) * LDK + 4 * (e & 7)]) = keep;
      *reinterpret_cast<float4*>(&Bs[cur ^ 1][(e >> 3) * LDK + 4 * (e & 7)]) = keep;
      *reinterpret_cast<float4*>(&As[cur ^ 1][((e + 256) >> 3) * LDK + 4 * (e & 7)]) = keep;
      *reinterpret_cast<float4*>(&Bs[cur ^ 1][((e + 256) >> 3) * LDK + 4 * (e & 7)]) = keep;
      __syncthreads();
    }
  }
  float t = 0;
  for (int i = 0; i < 16; ++i) t += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = t + keep.x;
}

template <int MODE>
void run(int occ) {
  const int steps = 2000, blocks = 256 * occ;
  float* out;
  (void)hipMalloc(&out, blocks * 256 * sizeof(float));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  probe<MODE><<<blocks, 256>>>(out, steps);
  (void)hipEventRecord(e0);
  probe<MODE><<<blocks, 256>>>(out, steps);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double fl = (double)blocks * 4 * steps * 16 * 4096.0;
  printf("mode %d (%s) occ %d: %.1f TF/s\n", MODE, MODE == 0 ? "lds+barrier" : MODE == 1 ? "lds reads" : "mfma only", occ,
         fl / (ms * 1e-3) / 1e12);
  (void)hipFree(out);
}

int main() {
  for (int o : {1, 2, 4}) { run<0>(o); run<1>(o); run<2>(o); }
  return 0;
}
