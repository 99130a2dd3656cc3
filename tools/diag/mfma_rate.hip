// Diagnostic only: back-to-back MFMA issue rate of v_mfma_f32_16x16x16_bf16 vs v_mfma_f32_16x16x32_bf16 (8 independent
// accumulators per wave, one wave per SIMD).  mfma_rate(kind, iters, out, stream): kind 0 = 16x16x16, 1 = 16x16x32;
// out[block] = a reduction of the accumulators (keeps the MFMAs live).  Time it with events on the host.
#include <hip/hip_runtime.h>
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void mfma_rate_kernel(int iters, float* out) {
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int l = threadIdx.x;
  s16x4 a4 = {(short)l, (short)(l + 1), (short)(l + 2), (short)(l + 3)};
  bf16x8 a8;
  for (int e = 0; e < 8; ++e) a8[e] = (__bf16)(0.001f * (l + e));
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (KIND == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, a4, acc[i], 0, 0, 0);
      else acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, a8, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.f) out[blockIdx.x] = s;
}

extern "C" int mfma_rate(int kind, int iters, float* out, int nblocks, hipStream_t stream) {
  if (kind == 0) mfma_rate_kernel<0><<<nblocks, 256, 0, stream>>>(iters, out);
  else mfma_rate_kernel<1><<<nblocks, 256, 0, stream>>>(iters, out);
  return (int)hipGetLastError();
}
