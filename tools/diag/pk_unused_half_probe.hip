// Does the UNUSED half of a packed-fp32 source pair change the result on gfx950?  (SLP repeatability investigation,
// DESIGN §6e.)  The SLP-vectorized twh_bwd splats a scalar with op_sel / op_sel_hi -- e.g. x2 - {Li, Li} becomes
//   v_pk_add_f32 v[d:d+1], v[x:x+1], v[l:l+1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]
// where v[l+1] is whatever the register last held (a bf16 fragment, a transcendental result, a permlane partner).
// ISA semantics say v[l+1] is not read.  This probe fills the unused half with special bit patterns (NaNs, infinities,
// denormals, huge values, random bits) and compares the hardware result bitwise with the scalar result.
//   hipcc --offload-arch=gfx950 -O2 tools/diag/pk_unused_half_probe.hip -o build/pk_unused_half_probe && build/pk_unused_half_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int NPAT = 10;
constexpr int NCASE = 5;

__device__ uint32_t pattern(int p, int lane) {
  switch (p) {
    case 0: return 0x3f800000u;                  // 1.0
    case 1: return 0x7fc00000u;                  // quiet NaN
    case 2: return 0x7f800001u;                  // signalling NaN
    case 3: return 0x7f800000u;                  // +inf
    case 4: return 0xff800000u;                  // -inf
    case 5: return 0x00000001u;                  // smallest denormal
    case 6: return 0x807fffffu;                  // largest negative denormal
    case 7: return 0x7f7fffffu;                  // FLT_MAX
    case 8: return 0x80000000u;                  // -0
    default: return 0x9e3779b9u * (lane + 7);    // random bits
  }
}

__global__ void probe(uint32_t* out) {
  const int lane = threadIdx.x;
  const float x0 = 0.37f + lane * 0.011f, x1 = -1.25f + lane * 0.007f, L = 3.5f - lane * 0.003f;
  for (int p = 0; p < NPAT; ++p) {
    const float junk = __builtin_bit_cast(float, pattern(p, lane));
    f2 x = {x0, x1};
    f2 l = {L, junk};
    f2 r0, r1, r2, r3, r4;
    // (a) x - {L, L} with L splatted from the lo half of l (the Li subtraction)
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r0) : "v"(x), "v"(l));
    // (b) x * L (splat) -- the pattern of the LOG2E / RoPE scalings
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r1) : "v"(x), "v"(l));
    // (c) fma(x, {L, L}, x) with the splat in src1
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r2) : "v"(x), "v"(l), "v"(x));
    // (d) src0 splat from the lo half of l: {L * x.lo, L * x.hi}
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r3) : "v"(l), "v"(x));
    // (e) SGPR pair with junk in the hi half (x * LOG2E + x with s[n:n+1] = {LOG2E, junk})
    const double sp = __builtin_bit_cast(double, f2{1.4426950408889634f, junk});
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r4) : "v"(x), "s"(sp), "v"(x));
    const float exp_[NCASE][2] = {{x0 - L, x1 - L},
                                  {x0 * L, x1 * L},
                                  {__builtin_fmaf(x0, L, x0), __builtin_fmaf(x1, L, x1)},
                                  {L * x0, L * x1},
                                  {__builtin_fmaf(x0, 1.4426950408889634f, x0), __builtin_fmaf(x1, 1.4426950408889634f, x1)}};
    const f2 got[NCASE] = {r0, r1, r2, r3, r4};
    for (int c = 0; c < NCASE; ++c)
      for (int h = 0; h < 2; ++h) {
        const int i = ((p * NCASE + c) * 2 + h) * 64 + lane;
        out[2 * i] = __builtin_bit_cast(uint32_t, h ? got[c].y : got[c].x);
        out[2 * i + 1] = __builtin_bit_cast(uint32_t, exp_[c][h]);
      }
  }
}

int main() {
  const int n = NPAT * NCASE * 2 * 64 * 2;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, n * sizeof(uint32_t)) != hipSuccess) return 2;
  probe<<<1, 64>>>(d);
  static uint32_t h[n];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
  const char* pn[NPAT] = {"1.0", "qNaN", "sNaN", "+inf", "-inf", "denorm+", "denorm-", "FLT_MAX", "-0", "random"};
  const char* cn[NCASE] = {"pk_add x-{L,L}", "pk_mul x*{L,L}", "pk_fma x*{L,L}+x", "pk_mul {L,L}*x (src0)",
                           "pk_fma SGPR pair"};
  int total = 0;
  for (int p = 0; p < NPAT; ++p)
    for (int c = 0; c < NCASE; ++c) {
      int bad = 0;
      for (int hh = 0; hh < 2; ++hh)
        for (int l = 0; l < 64; ++l) {
          const int i = ((p * NCASE + c) * 2 + hh) * 64 + l;
          bad += h[2 * i] != h[2 * i + 1];
        }
      total += bad;
      if (bad) printf("unused half %-8s %-24s mismatching results %d of 128\n", pn[p], cn[c], bad);
    }
  printf("total mismatches %d (of %d results)\n", total, NPAT * NCASE * 128);
  hipFree(d);
  return 0;
}
