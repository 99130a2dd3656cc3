// LDS access-pattern probe (gfx950): each kernel runs ONE lane -> address pattern of the fused attention kernels'
// head slices 4096 times per wave (16 waves per CU, every CU), so its time and its SQ_LDS_BANK_CONFLICT /
// SQ_LDS_IDX_ACTIVE counters (rocprofv3 --pmc, one kernel per pattern) show the LDS cycles that pattern costs.
// Checks tools/lds_banks.py's model (ds_write_b64 served in 4 x 16-lane groups on (dword mod 32) banks, ds_read_b128
// in 4 odd 16-lane groups, ds_read_b64_tr_b16 in 2 x 32 lanes, both on (dword mod 64) banks).
//   hipcc --offload-arch=gfx950 -O3 tools/lds_probe.hip -o tools/lds_probe && tools/lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// byte offset in a 16-row x 32-column bf16 head-slice region tile (two 16-column regions of 16 rows x 32 B) of
// element (r, c) under layout L:
//   0: region rows, 16-B halves swapped by bit 3 of the column XOR 1 (round 3, hs_off)
//   1: + 8-B slot XOR 2 * ((r >> 2) & 1)        (keeps 16-B pairs in order: ds_read_b128 unchanged)
//   2: + 8-B slot XOR ((r >> 2) & 3)            (16-B pairs swapped on odd rows groups)
//   3: 80-B plain rows (round 2, HLD = 40)
__device__ __forceinline__ int off(int L, int r, int c) {
  if (L == 3) return 2 * (r * 40 + c);
  const int region = c >> 4, cc = c & 15;
  int slot = cc >> 2;             // 8-B slot in the 32-B row
  slot ^= 2;                      // hs_off's constant half swap (bit 3 of the column XOR 1)
  if (L == 1) slot ^= 2 * ((r >> 2) & 1);
  if (L == 2) slot ^= (r >> 2) & 3;
  return region * 16 * 32 + r * 32 + slot * 8 + 2 * (cc & 3);
}

constexpr int ITERS = 4096;

// kind 0: ds_write_b64 of the MFMA D epilogue (lane (g, lr): row lr, cols 16t + 4g .. +3)
// kind 1: ds_read_b128 fragment (lane (g, lr): row lr, cols 8g .. 8g+7)
// kind 2: ds_read_b64_tr_b16 k-slot gather (lane (g, q, p): row 4g + q, cols 4p .. 4p+3)
template <int KIND, int L>
__global__ __launch_bounds__(256) void probe(float* out) {
  __shared__ __attribute__((aligned(16))) char lds[4][4096];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  char* base = lds[w];
  for (int i = lane; i < 1024; i += 64) reinterpret_cast<float*>(base)[i] = (float)i;
  __syncthreads();
  const int g = lane >> 4, lr = lane & 15;
  int a;
  if (KIND == 0) a = off(L, lr, 4 * g);
  else if (KIND == 1) a = off(L, lr, 8 * g);
  else a = off(L, 4 * g + ((lane >> 2) & 3), 4 * (lane & 3));
  float acc = 0.f;
  for (int it = 0; it < ITERS; ++it) {
    if (KIND == 0) {
      f32x2 v = {acc, (float)it};
      *reinterpret_cast<__attribute__((address_space(3))) f32x2*>((__attribute__((address_space(3))) char*)(base + a)) = v;
    } else if (KIND == 1) {
      const f32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(
          (const __attribute__((address_space(3))) char*)(base + a));
      acc += (v[0] + v[1]) + (v[2] + v[3]);
    } else {
      const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(base + a));
      acc += (float)(v[0] + v[1] + v[2] + v[3]);
    }
    asm volatile("" ::: "memory");
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int KIND, int L>
static float run(float* d, const char* name) {
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  probe<KIND, L><<<1024, 256>>>(d);
  (void)hipEventRecord(s);
  probe<KIND, L><<<1024, 256>>>(d);
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, s, e);
  printf("%-48s %8.1f us\n", name, ms * 1e3f);
  return ms;
}

int main() {
  float* d = nullptr;
  if (hipMalloc(&d, 1024 * 256 * sizeof(float)) != hipSuccess) return 2;
  run<0, 0>(d, "write_b64 epilogue, region (round 3)");
  run<0, 1>(d, "write_b64 epilogue, region + slot^2(r>>2&1)");
  run<0, 2>(d, "write_b64 epilogue, region + slot^(r>>2&3)");
  run<0, 3>(d, "write_b64 epilogue, 80-B rows (round 2)");
  run<1, 0>(d, "read_b128 fragment, region (round 3)");
  run<1, 1>(d, "read_b128 fragment, region + slot^2(r>>2&1)");
  run<1, 3>(d, "read_b128 fragment, 80-B rows (round 2)");
  run<2, 0>(d, "read_tr_b64 k-slot, region (round 3)");
  run<2, 1>(d, "read_tr_b64 k-slot, region + slot^2(r>>2&1)");
  run<2, 2>(d, "read_tr_b64 k-slot, region + slot^(r>>2&3)");
  run<2, 3>(d, "read_tr_b64 k-slot, 80-B rows (round 2)");
  (void)hipFree(d);
  return 0;
}
