// Fused temporal-attention block (bf16): Residual(PreNorm(EinopsToAndFrom(Attention)))
// (video_net.py:69-98, :350-454; rotary_embedding.py:29-48, :146-163; rel-pos bias :268-310):
//
//   y = x + W_out . attn( RoPE(scale * W_q LN(x)), RoPE(W_k LN(x)), W_v LN(x) ) + bias
//
// One block = P consecutive pixels of one sample x all F frames (F <= 16), V = P*F voxels.  The
// 768-channel qkv and the 256-channel attention output live only in LDS, one head at a time:
//   LN(x) -> xn (LDS) ; per head h:  [q|k|v]_h^T = W_h . xn^T (MFMA, RoPE + scale in the epilogue)
//   -> per pixel: S^T = K' Q'^T (one 16x16x32 MFMA, frames padded to 16) -> column softmax
//   (16-lane shuffles) -> O^T = V^T P^T (the S^T accumulator is the B operand directly: k-slot
//   (lane group g, element e<4) <-> key frame 4g+e) -> y^T += W_out[:, h] . O^T (MFMA).
// HBM traffic: x in, y out, LN stats and per-(voxel, head) log-sum-exp out — vs ~4 KB/voxel of
// qkv/o round trips for the unfused path.
#include "common.h"

namespace {

constexpr int NH = 8, DH = 32, INNER = 256, QKV = 768;
constexpr int HLD = 40;  // LDS row stride (bf16) of the per-head 32-wide tiles

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}

template <int C>
struct TB {
  static constexpr int P = 512 / C;       // pixels per block
  static constexpr int VPMAX = P * 16;    // rows when F == 16
  static constexpr int XLD = C + 8;       // xn row stride (bf16)
  static constexpr int L = C / 8;         // LN lanes per voxel
  static constexpr int CT = C / 16;       // 16-row output-channel tiles
  static constexpr int MAXT = (CT * (VPMAX / 16) + 3) / 4;
};

template <int C>
__global__ __launch_bounds__(256) void tblock_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ gamma,
                                                         const bf16* __restrict__ wqkv, const bf16* __restrict__ wout,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ rotg, bf16* __restrict__ y,
                                                         float* __restrict__ mr, float* __restrict__ lse, int F,
                                                         int HW, float scale, float eps) {
  using T = TB<C>;
  __shared__ __attribute__((aligned(16))) bf16 xn[T::VPMAX * T::XLD];
  __shared__ __attribute__((aligned(16))) bf16 sq[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 sk[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 sv[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 so[T::VPMAX * HLD];
  __shared__ float sb[NH * 16 * 16];
  __shared__ float rot[16 * 32];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * T::P;
  const int V = T::P * F;
  const int NV = (V + 15) >> 4;
  const int VP = NV * 16;

  for (int e = tid; e < NH * F * F; e += 256) {
    const int h = e / (F * F), r = e - h * F * F, i = r / F, j = r - i * F;
    sb[(h * 16 + i) * 16 + j] = bias[e];
  }
  for (int e = tid; e < F * 32; e += 256) rot[e] = rotg[e];

  // ---- LayerNorm (video_net.py:78-87) into LDS; rows >= V are zero
  {
    constexpr int VPP = 256 / T::L;
    const int sub = tid % T::L;
    for (int v0 = 0; v0 < VP; v0 += VPP) {
      const int v = v0 + tid / T::L;
      bool ok = false;
      int64_t row = 0;
      if (v < V) {
        const int pp = v / F, f = v - pp * F, p = p0 + pp;
        if (p < HW) { ok = true; row = ((int64_t)b * F + f) * HW + p; }
      }
      float a[8];
      if (ok) load8(x + row * C + sub * 8, a);
      else {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = 0.f;
      }
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s += a[i];
      s = group_sum(s, T::L);
      const float mean = s / C;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float d = a[i] - mean; q = fmaf(d, d, q); }
      q = group_sum(q, T::L);
      const float rstd = 1.f / sqrtf(q / C + eps);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = ok ? (a[i] - mean) * rstd * gamma[sub * 8 + i] : 0.f;
      if (v < VP) store8(xn + v * T::XLD + sub * 8, a);
      if (ok && sub == 0 && mr) { mr[row * 2] = mean; mr[row * 2 + 1] = rstd; }
    }
  }
  __syncthreads();

  f32x4 yacc[T::MAXT];
#pragma unroll
  for (int k = 0; k < T::MAXT; ++k) yacc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nty = T::CT * NV;

  for (int h = 0; h < NH; ++h) {
    // ---- [q|k|v]_h^T = W_h . xn^T ; tile (ct in 0..5, vt)
    for (int t = wid; t < 6 * NV; t += 4) {
      const int ct = t / NV, vt = t - ct * NV;
      const int kind = ct >> 1;
      const int wrow = kind * INNER + h * DH + (ct & 1) * 16 + lr;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < C; k0 += 32) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(wqkv + (int64_t)wrow * C + k0 + lg * 8);
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(xn + (vt * 16 + lr) * T::XLD + k0 + lg * 8);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc, 0, 0, 0);
      }
      const int v = vt * 16 + lr;
      const int f = v % F;
      const int d0 = (ct & 1) * 16 + lg * 4;
      float o4[4] = {acc[0], acc[1], acc[2], acc[3]};
      if (kind == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o4[r] *= scale;
      }
      if (kind < 2) {
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const int ri = (d0 >> 1) + pr;
          const float c = rot[f * 32 + ri * 2], s = rot[f * 32 + ri * 2 + 1];
          const float a0 = o4[2 * pr], a1 = o4[2 * pr + 1];
          o4[2 * pr] = a0 * c - a1 * s;
          o4[2 * pr + 1] = a1 * c + a0 * s;
        }
      }
      bf16* dst = kind == 0 ? sq : (kind == 1 ? sk : sv);
      store4(dst + v * HLD + d0, o4);
    }
    __syncthreads();
    // ---- attention core, one pixel per wave iteration
    for (int pp = wid; pp < T::P; pp += 4) {
      const int rb = pp * F;
      const bf16x8 ka = lr < F ? *reinterpret_cast<const bf16x8*>(sk + (rb + lr) * HLD + lg * 8) : zero8();
      const bf16x8 qb = lr < F ? *reinterpret_cast<const bf16x8*>(sq + (rb + lr) * HLD + lg * 8) : zero8();
      const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      // st[r] = S[i = lr][j = 4lg + r]
      float s[4];
      float m = -INFINITY;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = lg * 4 + r;
        s[r] = (j < F && lr < F) ? st[r] + sb[(h * 16 + lr) * 16 + j] : -INFINITY;
        m = fmaxf(m, s[r]);
      }
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      float pr[4], l = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pr[r] = s[r] == -INFINITY ? 0.f : expf(s[r] - m);
        l += pr[r];
      }
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
      const int p = p0 + pp;
      if (lse && lg == 0 && lr < F && p < HW) lse[(((int64_t)b * NH + h) * HW + p) * F + lr] = m + logf(l);
      const float inv = lr < F ? 1.f / l : 0.f;
      bf16x8 pb = zero8();
#pragma unroll
      for (int r = 0; r < 4; ++r) pb[r] = (bf16)(pr[r] * inv);
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        bf16x8 va = zero8();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = lg * 4 + r;
          if (j < F) va[r] = sv[(rb + j) * HLD + half * 16 + lr];
        }
        const f32x4 ot = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        // ot[r] = O[i = lr][d = half*16 + 4lg + r]
        if (lr < F) {
          float o4[4] = {ot[0], ot[1], ot[2], ot[3]};
          store4(so + (rb + lr) * HLD + half * 16 + lg * 4, o4);
        }
      }
    }
    __syncthreads();
    // ---- y^T += W_out[:, h*32:(h+1)*32] . O_h^T   (rows of `so` beyond V are never read as output)
#pragma unroll
    for (int k = 0; k < T::MAXT; ++k) {
      const int t = wid + 4 * k;
      if (t < nty) {
        const int ct = t / NV, vt = t - ct * NV;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(wout + (int64_t)(ct * 16 + lr) * INNER + h * DH + lg * 8);
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(so + (vt * 16 + lr) * HLD + lg * 8);
        yacc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, yacc[k], 0, 0, 0);
      }
    }
  }
  // ---- y = x + y_attn
#pragma unroll
  for (int k = 0; k < T::MAXT; ++k) {
    const int t = wid + 4 * k;
    if (t >= nty) continue;
    const int ct = t / NV, vt = t - ct * NV;
    const int v = vt * 16 + lr;
    if (v >= V) continue;
    const int pp = v / F, f = v - pp * F, p = p0 + pp;
    if (p >= HW) continue;
    const int64_t row = ((int64_t)b * F + f) * HW + p;
    const int co = ct * 16 + lg * 4;
    float xv[4];
    load4(x + row * C + co, xv);
    float o4[4] = {yacc[k][0] + xv[0], yacc[k][1] + xv[1], yacc[k][2] + xv[2], yacc[k][3] + xv[3]};
    store4(y + row * C + co, o4);
  }
}

}  // namespace

extern "C" {

// Fused forward of Residual(PreNorm(temporal Attention)): x,y [B*F*HW][C] bf16 (channels-last),
// wqkv [768][C] / wout [C][256] packed bf16, bias [8][F][F], rot [F][16][2].
// mr [B*F*HW][2] (LN mean, rstd) and lse [B][8][HW][F] are saved for the backward (may be null).
int cesm_tblock_fwd(const void* x, const float* gamma, const void* wqkv, const void* wout, const float* bias,
                    const float* rot, void* y, float* mr, float* lse, int B, int F, int HW, int C, float scale,
                    float eps, hipStream_t stream) {
  if (F < 1 || F > 16) return CESM_EUNSUPPORTED;
  switch (C) {
#define TB_CASE(CC)                                                                                            \
  case CC: {                                                                                                   \
    dim3 grid((unsigned)cdiv(HW, TB<CC>::P), B);                                                               \
    tblock_fwd_kernel<CC><<<grid, 256, 0, stream>>>((const bf16*)x, gamma, (const bf16*)wqkv, (const bf16*)wout, \
                                                    bias, rot, (bf16*)y, mr, lse, F, HW, scale, eps);          \
    break;                                                                                                     \
  }
    TB_CASE(64)
    TB_CASE(128)
    TB_CASE(256)
    TB_CASE(512)
#undef TB_CASE
    default:
      return CESM_EUNSUPPORTED;
  }
  return cesm_launch_status();
}

}  // extern "C"
