// Probe of the packed-fp32 VOP3P operand selection on gfx950 (the RoPE-epilogue repeatability investigation,
// DESIGN.md §2): each lane runs v_pk_mul_f32 / v_pk_fma_f32 with the op_sel / op_sel_hi / neg modifiers the SLP
// vectorizer emits for the rotation, on register pairs whose halves hold distinct sentinels, and stores what the
// hardware produced next to what the ISA semantics (LLVM's) predict.  Build + run:
//   hipcc --offload-arch=gfx950 -O2 tools/pk_probe.hip -o build/pk_probe && build/pk_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void probe(float* out) {
  const int l = threadIdx.x;
  const float base = 1.f + l;  // distinct per lane
  f2 a = {base * 1.f, base * 100.f};       // a.lo, a.hi
  f2 b = {2.f, 1000.f};                     // b.lo, b.hi
  f2 c = {3.f, 30000.f};                    // c.lo, c.hi
  f2 r0, r1, r2, r3, r4, r5, r6;
  // destination tied to a source pair whose LO half also feeds the HI result (op_sel_hi = 0): the SLP RoPE code
  // emits `v_pk_mul_f32 v[100:101], v[100:101], v[94:95] op_sel:[0,1] op_sel_hi:[0,0]`
  f2 t0 = a, t1 = b;
  asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[0,0]" : "+v"(t0) : "v"(b));
  asm volatile("v_pk_mul_f32 %0, %1, %0 op_sel:[1,0] op_sel_hi:[0,0]" : "+v"(t1) : "v"(a));
  // SGPR-pair operand (the SLP'd `x * LOG2E + b` reads its constant from s[n:n+1] with op_sel_hi:[1,0,1])
  const double sp = __builtin_bit_cast(double, f2{4.f, 7777.f});
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r5) : "v"(a), "s"(sp), "v"(c));
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r6) : "v"(a), "s"(sp));
  // the SLP RoPE pattern: lo = a.lo * b.hi, hi = a.lo * b.lo
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,0]" : "=v"(r0) : "v"(a), "v"(b));
  // lo = a.lo * b.lo - c.lo, hi = a.hi * b.hi - c.hi (neg on src2 both halves)
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[0,0,1] neg_hi:[0,0,1]" : "=v"(r1) : "v"(a), "v"(b), "v"(c));
  // lo = a.lo * b.lo + c.lo, hi = a.lo * b.hi + c.hi
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r2) : "v"(a), "v"(b), "v"(c));
  // default modifiers: lo = a.lo*b.lo, hi = a.hi*b.hi
  asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(r3) : "v"(a), "v"(b));
  // op_sel_hi:[1,0] on src1: hi = a.hi * b.lo
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r4) : "v"(a), "v"(b));
  const float exp_[18] = {a.x * b.y, a.x * b.x, a.x * b.x - c.x, a.y * b.y - c.y, a.x * b.x + c.x, a.x * b.y + c.y,
                          a.x * b.x, a.y * b.y, a.x * b.x, a.y * b.x,
                          a.x * 4.f + c.x, a.y * 4.f + c.y, a.x * 4.f, a.y * 4.f,
                          a.x * b.y, a.x * b.x, a.y * b.x, a.x * b.x};
  const float got[18] = {r0.x, r0.y, r1.x, r1.y, r2.x, r2.y, r3.x, r3.y, r4.x, r4.y, r5.x, r5.y, r6.x, r6.y,
                         t0.x, t0.y, t1.x, t1.y};
  for (int i = 0; i < 18; ++i) {
    out[(l * 18 + i) * 2] = got[i];
    out[(l * 18 + i) * 2 + 1] = exp_[i];
  }
}

int main() {
  float* d = nullptr;
  const int n = 64 * 18 * 2;
  if (hipMalloc(&d, n * sizeof(float)) != hipSuccess) return 2;
  probe<<<1, 64>>>(d);
  float h[n];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
  const char* names[18] = {"mul opsel[0,1] opselhi[0,0] lo", "                             hi",
                           "fma neg_lo/hi src2        lo", "                          hi",
                           "fma opselhi[0,1,1]        lo", "                          hi",
                           "mul default               lo", "                          hi",
                           "mul opselhi[1,0]          lo", "                          hi",
                           "fma SGPR src1 opselhi[1,0,1] lo", "                          hi",
                           "mul SGPR src1 opselhi[1,0] lo", "                          hi",
                           "mul dst=src0 opsel[0,1] hi[0,0] lo", "                          hi",
                           "mul dst=src1 opsel[1,0] hi[0,0] lo", "                          hi"};
  int bad = 0;
  for (int i = 0; i < 18; ++i) {
    int nb = 0;
    for (int l = 0; l < 64; ++l) nb += h[(l * 18 + i) * 2] != h[(l * 18 + i) * 2 + 1];
    bad += nb;
    printf("%-34s lane0 got %12.4f expected %12.4f  mismatching lanes %d\n", names[i], h[i * 2], h[i * 2 + 1], nb);
  }
  printf("total mismatches %d\n", bad);
  hipFree(d);
  return 0;
}
