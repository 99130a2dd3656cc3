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
#include "cesm_hip.h"
#include <type_traits>

namespace {

constexpr int NH = 8, DH = 32, INNER = 256, QKV = 768;
constexpr int HLD = 40;  // LDS row stride (bf16) of the per-head 32-wide tiles (tblock_*_kernel, C = 512)

// Per-head q / k / v / dO slices of the wave-private and head-parallel kernels (round 3): region tiles (common.h
// rg_off<1>) of two [R][16] regions -- head dims 0-15 and 16-31 -- with the two 16-B chunks of a row swapped when
// bit 2 of the row is set.  Pixel rows start at multiples of 4 (frames padded to F4 = pad4(F) rows), so the
// fragment reads of the attention core and the GEMMs, the k-slot gathers and the transposed dW reads are
// bank-conflict free and the bf16x4 epilogue stores 2-way (the minimum).  The round-2 80-B rows (HLD) were
// 2-way on the reads as well: 45-49 % of the LDS cycles of tw_fwd / twh_bwd were conflicts.
constexpr int HS = 32;  // bf16 per slice row (both regions)
template <int R>
__device__ __forceinline__ int hs_off(int r, int c) { return rg_off<1>(r, c, R * 16); }

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

// ============================================================================================
// Backward (dx path).  Per block: P_b pixels x F frames; loops over pixel groups (grid-stride) so
// the rel-pos-bias and LN-gamma gradient partials stay per block.  Per head h:
//   recompute [q'|k'|v]_h (as forward) and dO_h = dy . W_out[:, h]   (MFMA)
//   per pixel (MFMA, frames padded to 16):
//     S^T, P^T = exp(S^T + bias - lse), dP^T = V dO^T, D_i = sum_j P dP, dS^T = P^T (dP^T - D)
//     dQ'^T = K'^T dS^T ; O^T = V^T P^T ;  S, P, dP, dS (row-major orientation)
//     dK'^T = Q'^T dS ; dV^T = dO^T P       (k-slot trick: slot (g, e<4) <-> frame 4g+e)
//   dq = scale R^T dQ', dk = R^T dK' ; dxn += [dq|dk|dv] . W_qkv[h rows]   (MFMA, registers)
// then LN backward (+ residual dy) -> dx.  dqkv, O and xn are also written (bf16) for the two
// weight-gradient GEMMs.
// ============================================================================================
template <int C>
struct TBB {
  static constexpr int P = C >= 256 ? 1 : 256 / C;
  static constexpr int VPMAX = P * 16;
  static constexpr int XLD = C + 8;
  static constexpr int CT = C / 16;
  static constexpr int MAXT = (CT * (VPMAX / 16) + 3) / 4;
};

template <int C>
__global__ __launch_bounds__(256) void tblock_bwd_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, const float* __restrict__ gamma,
    const float* __restrict__ mr, const float* __restrict__ lse, const bf16* __restrict__ wqkv,
    const bf16* __restrict__ wqkv_t, const bf16* __restrict__ wout_t, const float* __restrict__ bias,
    const float* __restrict__ rotg, bf16* __restrict__ dx, bf16* __restrict__ dqkv_out, bf16* __restrict__ o_out,
    bf16* __restrict__ xn_out, float* __restrict__ dbias_part, float* __restrict__ dgamma_part, int F, int HW,
    float scale) {
  using T = TBB<C>;
  __shared__ __attribute__((aligned(16))) bf16 xn[T::VPMAX * T::XLD];
  __shared__ __attribute__((aligned(16))) bf16 dyl[T::VPMAX * T::XLD];
  __shared__ __attribute__((aligned(16))) bf16 sq[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 sk[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 sv[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 sdo[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 sdq[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 sdk[T::VPMAX * HLD];
  __shared__ __attribute__((aligned(16))) bf16 sdv[T::VPMAX * HLD];
  __shared__ float sb[NH * 16 * 16];
  __shared__ float rot[16 * 32];
  __shared__ float sLD[4][2][16];           // per wave: lse_i, D_i of the current pixel
  __shared__ float red[T::CT * T::VPMAX * 2];  // LN-bwd per-voxel partial sums
  __shared__ float sdb[NH * 16 * 16];        // block dbias accumulator (thread tid owns entries [h][tid])
  __shared__ float sdw[4 * 256];             // per-wave dbias of the current head
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int b = blockIdx.y;
  const int V = T::P * F;
  const int NV = (V + 15) >> 4;
  const int VP = NV * 16;
  const int npg = (HW + T::P - 1) / T::P;

  for (int e = tid; e < NH * F * F; e += 256) {
    const int h = e / (F * F), r = e - h * F * F, i = r / F, j = r - i * F;
    sb[(h * 16 + i) * 16 + j] = bias[e];
  }
  for (int e = tid; e < F * 32; e += 256) rot[e] = rotg[e];
  for (int e = tid; e < NH * 256; e += 256) sdb[e] = 0.f;

  float dgam[T::MAXT][4];
#pragma unroll
  for (int k = 0; k < T::MAXT; ++k)
#pragma unroll
    for (int r = 0; r < 4; ++r) dgam[k][r] = 0.f;
  const int nty = T::CT * NV;

  for (int pg = blockIdx.x; pg < npg; pg += gridDim.x) {
    const int p0 = pg * T::P;
    __syncthreads();  // previous group's LDS consumers done
    // ---- stage xn (LN with saved stats) and dy
    {
      constexpr int L = C / 8;
      constexpr int VPP = 256 / L;
      const int sub = tid % L;
      for (int v0 = 0; v0 < VP; v0 += VPP) {
        const int v = v0 + tid / L;
        bool ok = false;
        int64_t row = 0;
        if (v < V) {
          const int pp = v / F, f = v - pp * F, p = p0 + pp;
          if (p < HW) { ok = true; row = ((int64_t)b * F + f) * HW + p; }
        }
        float a[8], d[8];
        if (ok) {
          load8(x + row * C + sub * 8, a);
          load8(dy + row * C + sub * 8, d);
          const float mean = mr[row * 2], rstd = mr[row * 2 + 1];
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = (a[i] - mean) * rstd * gamma[sub * 8 + i];
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) { a[i] = 0.f; d[i] = 0.f; }
        }
        if (v < VP) {
          store8(xn + v * T::XLD + sub * 8, a);
          store8(dyl + v * T::XLD + sub * 8, d);
        }
        if (ok && xn_out) store8(xn_out + row * C + sub * 8, a);
      }
    }
    __syncthreads();

    f32x4 dxacc[T::MAXT];
#pragma unroll
    for (int k = 0; k < T::MAXT; ++k) dxacc[k] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int h = 0; h < NH; ++h) {
      // ---- recompute q',k',v (6 tiles per voxel tile) and dO_h (2 tiles)
      for (int t = wid; t < 8 * NV; t += 4) {
        const int ct = t / NV, vt = t - ct * NV;
        const int v = vt * 16 + lr;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if (ct < 6) {
          const int kind = ct >> 1;
          const int wrow = kind * INNER + h * DH + (ct & 1) * 16 + lr;
#pragma unroll
          for (int k0 = 0; k0 < C; k0 += 32) {
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(wqkv + (int64_t)wrow * C + k0 + lg * 8);
            const bf16x8 bb = *reinterpret_cast<const bf16x8*>(xn + v * T::XLD + k0 + lg * 8);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc, 0, 0, 0);
          }
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
          store4((kind == 0 ? sq : (kind == 1 ? sk : sv)) + v * HLD + d0, o4);
        } else {
          const int wrow = h * DH + (ct - 6) * 16 + lr;  // row of W_out^T [256][C]
#pragma unroll
          for (int k0 = 0; k0 < C; k0 += 32) {
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(wout_t + (int64_t)wrow * C + k0 + lg * 8);
            const bf16x8 bb = *reinterpret_cast<const bf16x8*>(dyl + v * T::XLD + k0 + lg * 8);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc, 0, 0, 0);
          }
          float o4[4] = {acc[0], acc[1], acc[2], acc[3]};
          store4(sdo + v * HLD + (ct - 6) * 16 + lg * 4, o4);
        }
      }
      __syncthreads();
      // ---- core backward per pixel
      float dbr[4] = {0.f, 0.f, 0.f, 0.f};
      for (int pp = wid; pp < T::P; pp += 4) {
        const int rb = pp * F;
        const int p = p0 + pp;
        const bool pix_ok = p < HW;
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
        const float Li = (lr < F && pix_ok) ? lse[(((int64_t)b * NH + h) * HW + p) * F + lr] : 0.f;
        // transposed orientation: lane col i = lr, rows j = 4lg + r
        const bf16x8 kr = lr < F ? *reinterpret_cast<const bf16x8*>(sk + (rb + lr) * HLD + lg * 8) : zero8();
        const bf16x8 qr = lr < F ? *reinterpret_cast<const bf16x8*>(sq + (rb + lr) * HLD + lg * 8) : zero8();
        const bf16x8 vr = lr < F ? *reinterpret_cast<const bf16x8*>(sv + (rb + lr) * HLD + lg * 8) : zero8();
        const bf16x8 dor = lr < F ? *reinterpret_cast<const bf16x8*>(sdo + (rb + lr) * HLD + lg * 8) : zero8();
        const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr, qr, z4, 0, 0, 0);    // S^T[j][i]
        const f32x4 dpt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vr, dor, z4, 0, 0, 0);  // dP^T[j][i]
        float pt[4], D = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = lg * 4 + r;
          const bool ok = j < F && lr < F;
          pt[r] = ok ? expf(st[r] + sb[(h * 16 + lr) * 16 + j] - Li) : 0.f;
          D = fmaf(pt[r], dpt[r], D);
        }
        D += __shfl_xor(D, 16, 64);
        D += __shfl_xor(D, 32, 64);
        if (lg == 0) { sLD[wid][0][lr] = Li; sLD[wid][1][lr] = D; }
        bf16x8 dst_b = zero8(), pt_b = zero8();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ds = pt[r] * (dpt[r] - D);
          dbr[r] += ds;
          dst_b[r] = (bf16)ds;
          pt_b[r] = (bf16)pt[r];
        }
        // dQ'^T[d][i] = sum_j K'[j][d] dS^T[j][i] ; O^T[d][i] = sum_j V[j][d] P^T[j][i]
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          bf16x8 ka = zero8(), va = zero8();
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = lg * 4 + r;
            if (j < F) {
              ka[r] = sk[(rb + j) * HLD + half * 16 + lr];
              va[r] = sv[(rb + j) * HLD + half * 16 + lr];
            }
          }
          const f32x4 dqt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, dst_b, z4, 0, 0, 0);
          const f32x4 ot = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pt_b, z4, 0, 0, 0);
          if (lr < F) {
            // dq = scale * R_i^T dQ'
            const int d0 = half * 16 + lg * 4;
            float o4[4] = {dqt[0], dqt[1], dqt[2], dqt[3]};
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
              const int ri = (d0 >> 1) + pr;
              const float c = rot[lr * 32 + ri * 2], s = -rot[lr * 32 + ri * 2 + 1];
              const float a0 = o4[2 * pr], a1 = o4[2 * pr + 1];
              o4[2 * pr] = (a0 * c - a1 * s) * scale;
              o4[2 * pr + 1] = (a1 * c + a0 * s) * scale;
            }
            store4(sdq + (rb + lr) * HLD + d0, o4);
            if (o_out && pix_ok) {
              float oo[4] = {ot[0], ot[1], ot[2], ot[3]};
              const int64_t row = ((int64_t)b * F + lr) * HW + p;
              store4(o_out + row * INNER + h * DH + d0, oo);
            }
          }
        }
        // row-major orientation: lane col j = lr, rows i = 4lg + r
        const f32x4 s_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qr, kr, z4, 0, 0, 0);   // S[i][j]
        const f32x4 dp_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dor, vr, z4, 0, 0, 0); // dP[i][j]
        bf16x8 ds_b = zero8(), p_b = zero8();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = lg * 4 + r;
          const bool ok = i < F && lr < F;
          const float pv = ok ? expf(s_[r] + sb[(h * 16 + i) * 16 + lr] - sLD[wid][0][i]) : 0.f;
          p_b[r] = (bf16)pv;
          ds_b[r] = (bf16)(ok ? pv * (dp_[r] - sLD[wid][1][i]) : 0.f);
        }
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          bf16x8 qa = zero8(), doa = zero8();
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = lg * 4 + r;
            if (i < F) {
              qa[r] = sq[(rb + i) * HLD + half * 16 + lr];
              doa[r] = sdo[(rb + i) * HLD + half * 16 + lr];
            }
          }
          const f32x4 dkt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, ds_b, z4, 0, 0, 0);   // dK'^T[d][j]
          const f32x4 dvt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(doa, p_b, z4, 0, 0, 0);   // dV^T[d][j]
          if (lr < F) {
            const int d0 = half * 16 + lg * 4;
            float o4[4] = {dkt[0], dkt[1], dkt[2], dkt[3]};
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
              const int ri = (d0 >> 1) + pr;
              const float c = rot[lr * 32 + ri * 2], s = -rot[lr * 32 + ri * 2 + 1];
              const float a0 = o4[2 * pr], a1 = o4[2 * pr + 1];
              o4[2 * pr] = a0 * c - a1 * s;
              o4[2 * pr + 1] = a1 * c + a0 * s;
            }
            store4(sdk + (rb + lr) * HLD + d0, o4);
            float v4[4] = {dvt[0], dvt[1], dvt[2], dvt[3]};
            store4(sdv + (rb + lr) * HLD + d0, v4);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sdw[wid * 256 + lr * 16 + lg * 4 + r] = dbr[r];
      __syncthreads();
      sdb[h * 256 + tid] += ((sdw[tid] + sdw[256 + tid]) + sdw[512 + tid]) + sdw[768 + tid];
      // ---- dxn^T += W_qkv^T[:, h cols] . dqkv_h^T ; also emit dqkv_h
#pragma unroll
      for (int k = 0; k < T::MAXT; ++k) {
        const int t = wid + 4 * k;
        if (t < nty) {
          const int ct = t / NV, vt = t - ct * NV;
          const int v = vt * 16 + lr;
#pragma unroll
          for (int kind = 0; kind < 3; ++kind) {
            const bf16* src = kind == 0 ? sdq : (kind == 1 ? sdk : sdv);
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(wqkv_t + (int64_t)(ct * 16 + lr) * QKV + kind * INNER +
                                                              h * DH + lg * 8);
            const bf16x8 bb = *reinterpret_cast<const bf16x8*>(src + v * HLD + lg * 8);
            dxacc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, dxacc[k], 0, 0, 0);
          }
        }
      }
      if (dqkv_out) {
        for (int e = tid; e < V * 12; e += 256) {   // V voxels x 3 kinds x 4 x 8-element chunks
          const int v = e / 12, rem = e - v * 12, kind = rem >> 2, part = rem & 3;
          const int pp = v / F, f = v - pp * F, p = p0 + pp;
          if (p >= HW) continue;
          const int64_t row = ((int64_t)b * F + f) * HW + p;
          const bf16* src = kind == 0 ? sdq : (kind == 1 ? sdk : sdv);
          *reinterpret_cast<bf16x8*>(dqkv_out + row * QKV + kind * INNER + h * DH + part * 8) =
              *reinterpret_cast<const bf16x8*>(src + v * HLD + part * 8);
        }
      }
      __syncthreads();  // sq/sk/sv/sdo/sdq/sdk/sdv reused by the next head
    }
    // ---- LN backward: g = dxn*gamma, dx = rstd*(g - mean(g) - xhat*mean(g*xhat)) + dy
#pragma unroll
    for (int k = 0; k < T::MAXT; ++k) {
      const int t = wid + 4 * k;
      float s1 = 0.f, s2 = 0.f;
      if (t < nty) {
        const int ct = t / NV, vt = t - ct * NV;
        const int v = vt * 16 + lr;
        bool ok = false;
        int64_t row = 0;
        if (v < V) {
          const int pp = v / F, f = v - pp * F, p = p0 + pp;
          if (p < HW) { ok = true; row = ((int64_t)b * F + f) * HW + p; }
        }
        const int co = ct * 16 + lg * 4;
        if (ok) {
          float xv[4];
          load4(x + row * C + co, xv);
          const float mean = mr[row * 2], rstd = mr[row * 2 + 1];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xh = (xv[r] - mean) * rstd;
            const float g = dxacc[k][r] * gamma[co + r];
            s1 += g;
            s2 = fmaf(g, xh, s2);
            dgam[k][r] = fmaf(dxacc[k][r], xh, dgam[k][r]);
          }
        }
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (lg == 0) { red[(ct * T::VPMAX + v) * 2] = s1; red[(ct * T::VPMAX + v) * 2 + 1] = s2; }
      }
    }
    __syncthreads();
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
      float S1 = 0.f, S2 = 0.f;
      for (int c2 = 0; c2 < T::CT; ++c2) { S1 += red[(c2 * T::VPMAX + v) * 2]; S2 += red[(c2 * T::VPMAX + v) * 2 + 1]; }
      S1 /= C;
      S2 /= C;
      const float mean = mr[row * 2], rstd = mr[row * 2 + 1];
      const int co = ct * 16 + lg * 4;
      float xv[4], o4[4];
      load4(x + row * C + co, xv);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float xh = (xv[r] - mean) * rstd;
        o4[r] = rstd * (dxacc[k][r] * gamma[co + r] - S1 - xh * S2) + (float)dyl[v * T::XLD + co + r];
      }
      store4(dx + row * C + co, o4);
    }
  }
  // ---- block partials: dbias -> relpos layout [b][h][blk][F][F]
  __syncthreads();
  for (int e = tid; e < NH * F * F; e += 256) {
    const int h = e / (F * F), r = e - h * F * F, i = r / F, j = r - i * F;
    dbias_part[(((int64_t)b * NH + h) * gridDim.x + blockIdx.x) * F * F + r] = sdb[(h * 16 + i) * 16 + j];
  }
  // dgamma: reduce each lane's per-channel partials over the 16 voxel lanes, then tiles/waves in order
#pragma unroll
  for (int k = 0; k < T::MAXT; ++k)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) dgam[k][r] += __shfl_xor(dgam[k][r], o, 64);
  float* sg = red;  // reuse: C floats
  for (int e = tid; e < C; e += 256) sg[e] = 0.f;
  __syncthreads();
  for (int w = 0; w < 4; ++w) {
    if (wid == w && lr == 0) {
#pragma unroll
      for (int k = 0; k < T::MAXT; ++k) {
        const int t = wid + 4 * k;
        if (t < nty) {
          const int ct = t / NV;
#pragma unroll
          for (int r = 0; r < 4; ++r) sg[ct * 16 + lg * 4 + r] += dgam[k][r];
        }
      }
    }
    __syncthreads();
  }
  for (int e = tid; e < C; e += 256) dgamma_part[((int64_t)b * gridDim.x + blockIdx.x) * C + e] = sg[e];
}

// ============================================================================================
// Wave-private variants (C <= 256).  Each wave owns PW consecutive pixels x F frames (VW = PW*F
// voxels, NVT = ceil(VW/16) voxel tiles) end to end, so there are no block barriers after the
// table preload:
//   * LN is evaluated on the MFMA B fragments in registers (lane (g, r): voxel r of the tile,
//     channels ks*32 + 8g..8g+7); per-voxel sums via 16/32-lane shuffles;
//   * per head, [q'|k'|v] (and dO in the backward) go to a wave-private LDS slice of NVT*16 rows;
//   * each weight fragment is loaded once per head and reused for all NVT voxel tiles.
// ============================================================================================
template <int C, int NV = 1>
struct TW {
  static constexpr int PW = C <= 64 ? 4 : (C == 128 ? 2 : 1);  // pixels per wave
  static constexpr int KS = C / 32;                            // k-steps of the C-deep GEMMs
  static constexpr int CT = C / 16;                            // 16-channel output tiles
  static constexpr int NVTM = NV;                              // voxel tiles of the wave (<= PW)
};

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ bf16x8 ld16(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// sum / max over the 4 lanes {l, l^16, l^32, l^48} with v_permlane{16,32}_swap (VALU, no LDS)
__device__ __forceinline__ float grp4_sum(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float grp4_max(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

constexpr int RS = 36;  // RoPE table row stride (floats): 16-B aligned, spreads frames over banks
constexpr float LOG2E = 1.4426950408889634f;

// k-slot gather with the hardware transpose read: lane (g, i) gets tile[rb + 4g + e][c0 + i] in
// element e (e < 4; elements 4..7 and rows >= F are zero).  Must run with EXEC all ones.
// (tile: a head slice of R rows, hs_off layout; rb % 4 == 0)
template <int R>
__device__ __forceinline__ bf16x8 kslot_gather(const bf16* tile, int rb, int c0, int F, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + rg_at(rb, hs_off<R>(4 * g + q, c0 + 4 * p))));
  bf16x8 r = zero8();
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (4 * g + e < F) r[e] = __builtin_bit_cast(bf16, (short)v[e]);
  return r;
}

// kslot_gather<R> without the per-element frame mask (see kslot_raw): for operands whose partner is zero at every
// k-slot of a frame >= F
__device__ __forceinline__ bf16x8 kslot_raw(const s16x4 v) {
  bf16x8 r = zero8();
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = __builtin_bit_cast(bf16, (short)v[e]);
  return r;
}
template <int R>
__device__ __forceinline__ bf16x8 kslot_gather_raw(const bf16* tile, int rb, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  return kslot_raw(__builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + rg_at(rb, hs_off<R>(4 * g + q, c0 + 4 * p)))));
}

// The attention-core products over frames (P V, dS K, dS^T Q, P^T dO) have K = 16 frames: they run as
// v_mfma_f32_16x16x16_bf16 on 4-element operands -- the k-slot gather's hardware-transpose result as it comes, P /
// dS packed from the lane's 4 score entries -- half the MFMA cycles of the 16x16x32 form with slots 4..7 zeroed,
// and no zero fill moves.  Slot (g, e) pairs the same entries in both forms.
__device__ __forceinline__ f32x4 mfma_k16(const s16x4 a, const s16x4 b, const f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ s16x4 bf16x4_bits(float a, float b, float c, float d) {
  const bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  return __builtin_bit_cast(s16x4, v);
}
template <int R>
__device__ __forceinline__ s16x4 kslot4(const bf16* tile, int rb, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + rg_at(rb, hs_off<R>(4 * g + q, c0 + 4 * p))));
}

// hardware-transpose read of a head slice: lane (g, i) <- tile[r0 + 4g + e][c0 + i]
template <int R>
__device__ __forceinline__ s16x4 tr4_hs(const bf16* tile, int r0, int c0, int lane) {
  return tr4_rg<1>(tile, r0, c0, R * 16, lane);
}

// RoPE rotation of 4 consecutive head dims d0..d0+3 (two pairs) of frame f; sign=-1 applies R^T
__device__ __forceinline__ void rope4(float* o4, const float* rot, int f, int d0, float sign) {
  const f32x4 cs = *reinterpret_cast<const f32x4*>(rot + f * RS + d0);  // (c0, s0, c1, s1)
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    const float c = cs[2 * pr], sn = sign * cs[2 * pr + 1];
    const float a0 = o4[2 * pr], a1 = o4[2 * pr + 1];
    o4[2 * pr] = a0 * c - a1 * sn;
    o4[2 * pr + 1] = a1 * c + a0 * sn;
  }
}

__device__ __forceinline__ bf16x8 sel8(bool ok, bf16x8 v) { return ok ? v : zero8(); }

// rows of voxel v of the wave's pixel group
// (slice rows: pixel pp's frames at rows pp*F4 + f, F4 = F rounded up to a multiple of 4, VW = PW*F4; rows with
// f >= F are padding.  Every pixel's rows then start on a multiple of 4, which the hs_off layout needs for its
// conflict-free reads and which lets the address of row rb + i split into a per-lane part and a uniform XOR.)
__device__ __forceinline__ int pad4(int F) { return (F + 3) & ~3; }
__device__ __forceinline__ bool tw_row(int v, int VW, int F, int F4, int p0, int HW, int b, int64_t& row) {
  if (v >= VW) return false;
  const int pp = v / F4, f = v - pp * F4, p = p0 + pp;
  if (f >= F || p >= HW) return false;
  row = ((int64_t)b * F + f) * HW + p;
  return true;
}

// q'|k'|v tiles (and the RoPE/scale epilogue) of head h for the wave's NVT voxel tiles
template <int C, int NV>
__device__ __forceinline__ void tw_load_wq(bf16x8 (&a)[6][C / 32], const bf16* __restrict__ wqkv, int h, int lr,
                                           int lg) {
  // wqkv = A-fragment image of W_qkv [768][C] (frag_image): 1-KiB line per fragment
#pragma unroll
  for (int ct = 0; ct < 6; ++ct) {
    const int mt = (ct >> 1) * 16 + h * 2 + (ct & 1);
#pragma unroll
    for (int ks = 0; ks < TW<C, NV>::KS; ++ks) a[ct][ks] = ld_img(wqkv, mt, TW<C, NV>::KS, ks, lg * 16 + lr);
  }
}

// q'|k'|v tiles (RoPE/scale epilogue) of one head from preloaded weight fragments a[6][KS]
template <int C, int NV>
__device__ __forceinline__ void tw_qkv_pre(const bf16x8 (&a)[6][C / 32],
                                           const bf16x8 (&xf)[TW<C, NV>::NVTM][TW<C, NV>::KS], const int (&fr)[NV],
                                           float scale, const float* rot, bf16* sq, bf16* sk, bf16* sv, int lr, int lg) {
  using T = TW<C, NV>;
  constexpr int R = NV * 16;  // slice rows
#pragma unroll
  for (int ct = 0; ct < 6; ++ct) {
    const int kind = ct >> 1;
    bf16* dst = kind == 0 ? sq : (kind == 1 ? sk : sv);
    const int d0 = (ct & 1) * 16 + lg * 4;
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ct][ks], xf[vt][ks], acc, 0, 0, 0);
      float o4[4] = {acc[0], acc[1], acc[2], acc[3]};
      if (kind == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o4[r] *= scale;
      }
      if (kind < 2) rope4(o4, rot, fr[vt], d0, 1.f);
      store4(dst + hs_off<R>(vt * 16 + lr, d0), o4);
    }
  }
}

template <int C, int NV, bool FULL = (C <= 64)>
__device__ __forceinline__ void tw_qkv(const bf16* __restrict__ wqkv, const bf16x8 (&xf)[TW<C, NV>::NVTM][TW<C, NV>::KS],
                                       int h, const int (&fr)[NV], float scale, const float* rot, bf16* sq, bf16* sk,
                                       bf16* sv, int lr, int lg) {
  constexpr int R = NV * 16;  // slice rows
  if constexpr (FULL) {
    bf16x8 a[6][C / 32];
    tw_load_wq<C, NV>(a, wqkv, h, lr, lg);
    tw_qkv_pre<C, NV>(a, xf, fr, scale, rot, sq, sk, sv, lr, lg);
  } else {
    // wider C: the six 16-row tiles' fragments (24 x 16 B at C = 128) in two-tile batches, which keeps
    // the backward kernel within its 256 registers
    using T = TW<C, NV>;
#pragma unroll
    for (int c2 = 0; c2 < 6; c2 += 2) {
      bf16x8 a[2][T::KS];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int ct = c2 + u, mt = (ct >> 1) * 16 + h * 2 + (ct & 1);
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) a[u][ks] = ld_img(wqkv, mt, T::KS, ks, lg * 16 + lr);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int ct = c2 + u, kind = ct >> 1;
        bf16* dst = kind == 0 ? sq : (kind == 1 ? sk : sv);
        const int d0 = (ct & 1) * 16 + lg * 4;
#pragma unroll
        for (int vt = 0; vt < NV; ++vt) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < T::KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][ks], xf[vt][ks], acc, 0, 0, 0);
          float o4[4] = {acc[0], acc[1], acc[2], acc[3]};
          if (kind == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o4[r] *= scale;
          }
          if (kind < 2) rope4(o4, rot, fr[vt], d0, 1.f);
          store4(dst + hs_off<R>(vt * 16 + lr, d0), o4);
        }
      }
    }
  }
}

// RoPE of dims d0..d0+3 (two pairs) with preloaded coefficients cs = (c0, s0, c1, s1)
__device__ __forceinline__ void rope4c(float* o4, const f32x4 cs) {
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    const float c = cs[2 * pr], sn = cs[2 * pr + 1];
    const float a0 = o4[2 * pr], a1 = o4[2 * pr + 1];
    o4[2 * pr] = a0 * c - a1 * sn;
    o4[2 * pr + 1] = a1 * c + a0 * sn;
  }
}
// q'|k'|v tiles of one head, batched per kind (round 4): the kind's 2 x NV tiles (independent accumulators) are
// issued back to back, the next kind's weight fragments are in flight meanwhile (double buffer), and the RoPE
// coefficients are read from LDS before the MFMAs, so the epilogue waits on nothing.  (Round 3 ran each tile as
// load-wait -> 2 MFMAs -> s_nop -> LDS read -> wait -> VALU -> store, one chain at a time.)
template <int C, int NV, bool QSCALE = true>
__device__ __forceinline__ void tw_qkv_b(const bf16* __restrict__ wqkv, const bf16x8 (&xf)[NV][C / 32], int h,
                                         const int (&fr)[NV], float scale, const float* rot, bf16* sq, bf16* sk,
                                         bf16* sv, int lr, int lg) {
  using T = TW<C, NV>;
  constexpr int R = NV * 16;
  // 6 (kind, half) column tiles; the next tile's weight fragments in flight while this one computes
  bf16x8 a[2][T::KS];
  auto ld = [&](int ct, int buf) {
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks) a[buf][ks] = ld_img(wqkv, (ct >> 1) * 16 + h * 2 + (ct & 1), T::KS, ks, lg * 16 + lr);
  };
  ld(0, 0);
#pragma unroll
  for (int ct = 0; ct < 6; ++ct) {
    const int buf = ct & 1, kind = ct >> 1, u = ct & 1;
    if (ct + 1 < 6) ld(ct + 1, buf ^ 1);
    f32x4 cs[NV];
    if (kind < 2) {
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) cs[vt] = *reinterpret_cast<const f32x4*>(rot + fr[vt] * RS + u * 16 + lg * 4);
    }
    f32x4 acc[NV];
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      acc[vt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) acc[vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[buf][ks], xf[vt][ks], acc[vt], 0, 0, 0);
    }
    bf16* dst = kind == 0 ? sq : (kind == 1 ? sk : sv);
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      float o4[4] = {acc[vt][0], acc[vt][1], acc[vt][2], acc[vt][3]};
      if (QSCALE && kind == 0) {  // (folded weights: the scale is in the q rows)
#pragma unroll
        for (int r = 0; r < 4; ++r) o4[r] *= scale;
      }
      if (kind < 2) rope4c(o4, cs[vt]);
      store4(dst + hs_off<R>(vt * 16 + lr, u * 16 + lg * 4), o4);
    }
  }
}

// LN of the wave's voxels on the B fragments.  use_saved: take (mean, rstd) from mr, else compute
// them (and store them to mr when non-null).
template <int C, int NV, bool GAM = true>
__device__ __forceinline__ void tw_ln(const bf16* __restrict__ x, const float* __restrict__ gamma, float* mr_out,
                                      const float* __restrict__ mr_in, bf16x8 (&xf)[TW<C, NV>::NVTM][TW<C, NV>::KS], int NVT,
                                      int VW, int F, int F4, int p0, int HW, int b, float eps, int lr, int lg) {
  using T = TW<C, NV>;
  // every load is unconditional (invalid voxels read row 0 and are zeroed by a select): a load under a
  // lane predicate becomes a branch with its own vmcnt(0), which serialised the 16 gamma and 2 x loads
  // of every voxel tile
  float gm[T::KS][8];
#pragma unroll
  for (int ks = 0; ks < T::KS; ++ks) {
    if constexpr (GAM) load8(gamma + ks * 32 + lg * 8, gm[ks]);
    else
#pragma unroll
      for (int i = 0; i < 8; ++i) gm[ks][i] = 1.f;  // gamma folded into the weights (xf = xhat)
  }
  bf16x8 raw[T::NVTM][T::KS];
  bool okv[T::NVTM];
  int64_t rows[T::NVTM];
#pragma unroll
  for (int vt = 0; vt < T::NVTM; ++vt) {
    int64_t row = 0;
    okv[vt] = vt < NVT && tw_row(vt * 16 + lr, VW, F, F4, p0, HW, b, row);
    rows[vt] = okv[vt] ? row : 0;
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks) raw[vt][ks] = ld16(x + rows[vt] * C + ks * 32 + lg * 8);
  }
#pragma unroll
  for (int vt = 0; vt < T::NVTM; ++vt) {
    const bool ok = okv[vt];
    float a[T::KS][8];
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i) a[ks][i] = ok ? (float)raw[vt][ks][i] : 0.f;
    float mean, rstd;
    if (mr_in) {
      const float m0 = mr_in[rows[vt] * 2], r0 = mr_in[rows[vt] * 2 + 1];
      mean = ok ? m0 : 0.f;
      rstd = ok ? r0 : 0.f;
    } else {
      float s = 0.f;
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks)
#pragma unroll
        for (int i = 0; i < 8; ++i) s += a[ks][i];
      s = grp4_sum(s);
      mean = s / C;
      float q = 0.f;
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks)
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float d = a[ks][i] - mean; q = fmaf(d, d, q); }
      q = grp4_sum(q);
      rstd = 1.f / sqrtf(q / C + eps);
      if (ok && lg == 0 && mr_out) { mr_out[rows[vt] * 2] = mean; mr_out[rows[vt] * 2 + 1] = rstd; }
    }
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i) xf[vt][ks][i] = (bf16)(ok ? (a[ks][i] - mean) * rstd * gm[ks][i] : 0.f);
  }
}

// waves per SIMD of tw_fwd: at C = 64 LDS-bound (per-wave q/k/v slices + tables: 3 blocks of 53 KB);
// at C >= 128 register-bound (the out-projection accumulators spill below 256 VGPRs)
typedef unsigned int tw_u32x2 __attribute__((ext_vector_type(2)));
// Measured and removed (profiles/r5f_tw_fwd_lse_late_tb.txt, r5f_epilogue_loads_first_tb.txt, r2_v13_*): the next
// head's first weight tile loaded before the O stores (21 spilled registers, +5 %), every residual load before the y
// stores (4 spills, +1-3 %), 2 waves per SIMD with the next head's weights prefetched in registers (+2 %), pixels
// interleaved phase by phase in the attention core (neutral).
template <int C>
constexpr int tw_fwd_occ() { return C <= 64 ? 3 : 2; }
template <int C, int NV, bool FOLD = false>
__global__ __launch_bounds__(256, tw_fwd_occ<C>()) void tw_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ gamma,
                                                     const bf16* __restrict__ wqkv, const bf16* __restrict__ wout,
                                                     const float* __restrict__ bias, const float* __restrict__ rotg,
                                                     bf16* __restrict__ y, float* __restrict__ mr,
                                                     float* __restrict__ lse, bf16* __restrict__ o_out, int F, int HW,
                                                     float scale, float eps) {
  using T = TW<C, NV>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sb = smem;                              // [8][F][F], pre-scaled by log2(e)
  float* rot = smem + ((NH * F * F + 3) & ~3);   // [16][RS]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int b = blockIdx.y;
  const int F4 = pad4(F), VW = T::PW * F4;
  constexpr int NVT = NV;
  const int R = NVT * 16;
  bf16* sq = reinterpret_cast<bf16*>(rot + 16 * RS) + wid * 3 * R * HS;
  bf16* sk = sq + R * HS;
  bf16* sv = sk + R * HS;
  for (int e = tid; e < NH * F * F; e += 256) sb[e] = bias[e] * LOG2E;
  for (int e = tid; e < F * 32; e += 256) rot[(e >> 5) * RS + (e & 31)] = rotg[e];
  // tail pad past the last wave's slices: its last pixel's unmasked V gathers read up to 16 - F4 <= 12 rows into it
  for (int e = tid; e < 256; e += 256) reinterpret_cast<float*>(reinterpret_cast<bf16*>(rot + 16 * RS) + 4 * 3 * R * HS)[e] = 0.f;
  const int p0 = (blockIdx.x * 4 + wid) * T::PW;
  // a wave without pixels (the last block when cdiv(HW, PW) is not a multiple of 4) zeroes its q rows before it
  // leaves: the previous wave's last pixel gathers up to 12 rows past its own slices, i.e. into this wave's q rows,
  // which must be finite (P^T is 0 there, but 0 x a stale Inf / NaN pattern left by an earlier kernel is NaN; found by
  // tools/vgpr_pollute_check.py at HW = 4: one pixel's y non-finite, depending on the LDS contents)
  if (p0 >= HW)
    for (int e = lane; e < R * HS / 8; e += 64) reinterpret_cast<bf16x8*>(sq)[e] = zero8();
  __syncthreads();
  if (p0 >= HW) return;
  int fr[NV];
#pragma unroll
  for (int vt = 0; vt < NV; ++vt) fr[vt] = (vt * 16 + lr) % F4 < F ? (vt * 16 + lr) % F4 : 0;

  bf16x8 xf[T::NVTM][T::KS];
  // FOLD: wqkv is the image of W diag(gamma) and the B fragments hold xhat (twh_bwd_kernel recomputes
  // q/k/v the same way, so forward and backward see identical bf16 operands)
  tw_ln<C, NV, !FOLD>(x, gamma, mr, nullptr, xf, NVT, VW, F, F4, p0, HW, b, eps, lr, lg);

  f32x4 yacc[T::CT][T::NVTM];
#pragma unroll
  for (int ct = 0; ct < T::CT; ++ct)
#pragma unroll
    for (int vt = 0; vt < T::NVTM; ++vt) yacc[ct][vt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};

  // C = 64: the head's lse stored after the to_out weight loads (vmcnt counts loads and stores in order: a load
  // issued after a store also waits for it; round 5 -0.8 %)
  constexpr bool LE = C == 64;
  for (int h = 0; h < NH; ++h) {
    bf16x8 wo[T::CT];
    if constexpr (C == 64) tw_qkv_b<C, NV, !FOLD>(wqkv, xf, h, fr, scale, rot, sq, sk, sv, lr, lg);
    else tw_qkv<C, NV, false>(wqkv, xf, h, fr, FOLD ? 1.f : scale, rot, sq, sk, sv, lr, lg);  // two-tile batches
    // bias (log2 units) of this lane's 4 entries (i = lr, j = 4g + r); -inf masks padding frames
    float bt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = lg * 4 + r;
      // query lanes lr >= F take row 0's biases: their max is finite, so no lane needs a -inf guard below (their
      // O columns and lse are never stored)
      bt[r] = j < F ? sb[(h * F + (lr < F ? lr : 0)) * F + j] : -INFINITY;
    }
    wave_lds_sync();
    // attention core, base-2 softmax; O overwrites the pixel's own q rows.  Pixels go in groups of PG
    // with each phase issued for the whole group (independent MFMA -> softmax -> MFMA chains
    // interleave instead of serialising on the MFMA result latency).  Pixels past HW hold zero rows
    // (their LN input is masked): computing them is harmless, only the lse store is guarded.
    constexpr int PG = 1;  // (2 / 4 measured neutral)
    float lsev[T::PW];  // LE: the pixels' lse (log2 units)
#pragma unroll
    for (int pg = 0; pg < T::PW; pg += PG) {
      f32x4 st[PG];
#pragma unroll
      for (int u = 0; u < PG; ++u) {
        const int rb = (pg + u) * F4;
        // rows past F read the pixel's row 0 (finite): key rows j >= F are masked by bt = -inf below and query
        // columns i >= F are never stored, so no select is needed
        const int rr = rg_at(rb, hs_off<R>(lr < F ? lr : 0, lg * 8));
        const bf16x8 ka = ld16(sk + rr);
        const bf16x8 qb = ld16(sq + rr);
        st[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qb, z4, 0, 0, 0);
      }
      s16x4 va[PG][2];
#pragma unroll
      for (int u = 0; u < PG; ++u)
#pragma unroll
        for (int half = 0; half < 2; ++half) va[u][half] = kslot4<R>(sv, (pg + u) * F4, half * 16, lane);  // P^T is 0 at keys >= F
      s16x4 pb[PG];
#pragma unroll
      for (int u = 0; u < PG; ++u) {
        const int p = p0 + pg + u;
        float sc[4];
        float m = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sc[r] = fmaf(st[u][r], LOG2E, bt[r]);
          m = fmaxf(m, sc[r]);
        }
        m = grp4_max(m);
        float pr[4], l = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pr[r] = __builtin_amdgcn_exp2f(sc[r] - m);  // exp2(-inf) = 0 past F (m is finite: key 0 < F)
          l += pr[r];
        }
        l = grp4_sum(l);
        if (LE) lsev[pg + u] = m + log2f(l);  // stored after the to_out weight loads
        else if (lse && lg == 0 && lr < F && p < HW) lse[(((int64_t)b * NH + h) * HW + p) * F + lr] = m + log2f(l);  // log2 units
        const float inv = __builtin_amdgcn_rcpf(l);
        pb[u] = bf16x4_bits(pr[0] * inv, pr[1] * inv, pr[2] * inv, pr[3] * inv);
      }
#pragma unroll
      for (int u = 0; u < PG; ++u) {
        const int rb = (pg + u) * F4;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const f32x4 ot = mfma_k16(va[u][half], pb[u], z4);
          if (lr < F) {
            float o4[4] = {ot[0], ot[1], ot[2], ot[3]};
            store4(sq + rg_at(rb, hs_off<R>(lr, half * 16 + lg * 4)), o4);
          }
        }
      }
    }
    {  // issued after the core: keeps the 16 registers out of the qkv phase
#pragma unroll
      for (int ct = 0; ct < T::CT; ++ct) wo[ct] = ld_img(wout, ct, INNER / 32, h, lane);
    }
    if constexpr (LE) {
      __builtin_amdgcn_sched_barrier(0);
      if (lse && lg == 0 && lr < F) {
#pragma unroll
        for (int u = 0; u < T::PW; ++u)
          if (p0 + u < HW) lse[(((int64_t)b * NH + h) * HW + p0 + u) * F + lr] = lsev[u];
      }
    }
    wave_lds_sync();
    // y^T += W_out[:, h] . O_h^T
    bf16x8 ob[T::NVTM];
#pragma unroll
    for (int vt = 0; vt < T::NVTM; ++vt) ob[vt] = vt < NVT ? ld16(sq + hs_off<R>(vt * 16 + lr, lg * 8)) : zero8();
    if (o_out) {  // O_h for the to_out weight gradient (the backward then skips its emission)
#pragma unroll
      for (int vt = 0; vt < T::NVTM; ++vt) {
        int64_t row = 0;
        if (vt < NVT && tw_row(vt * 16 + lr, VW, F, F4, p0, HW, b, row))
          stnt16(o_out + row * INNER + h * DH + lg * 8, ob[vt]);
      }
    }
#pragma unroll
    for (int ct = 0; ct < T::CT; ++ct) {
#pragma unroll
      for (int vt = 0; vt < T::NVTM; ++vt)
        if (vt < NVT) yacc[ct][vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wo[ct], ob[vt], yacc[ct][vt], 0, 0, 0);
    }
    wave_lds_sync();
  }
  // y = x + attn
#pragma unroll
  for (int vt = 0; vt < T::NVTM; ++vt) {
    if (vt >= NVT) break;
    int64_t row = 0;
    if (!tw_row(vt * 16 + lr, VW, F, F4, p0, HW, b, row)) continue;
#pragma unroll
    for (int ct = 0; ct < T::CT; ++ct) {
      const int co = ct * 16 + lg * 4;
      float xv[4];
      load4(x + row * C + co, xv);
      float o4[4] = {yacc[ct][vt][0] + xv[0], yacc[ct][vt][1] + xv[1], yacc[ct][vt][2] + xv[2], yacc[ct][vt][3] + xv[3]};
      store4(y + row * C + co, o4);
    }
  }
}

template <int C, int NV>
__global__ __launch_bounds__(256, 2) void tw_bwd_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, const float* __restrict__ gamma,
    const float* __restrict__ mr, const float* __restrict__ lse, const bf16* __restrict__ wqkv,
    const bf16* __restrict__ wqkv_t, const bf16* __restrict__ wout_t, const float* __restrict__ bias,
    const float* __restrict__ rotg, bf16* __restrict__ dx, bf16* __restrict__ dqkv_out, bf16* __restrict__ o_out,
    bf16* __restrict__ xn_out, float* __restrict__ dbias_part, float* __restrict__ dgamma_part, int F, int HW,
    float scale) {
  using T = TW<C, NV>;
  constexpr bool DG_REG = false;  // dgamma partials flushed per pixel group (LDS atomics)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int FF = F * F;
  // dbias / dgamma accumulators per wave ([4][8][F][F], [4][C]; one writer each, summed in a fixed order at the
  // end, so the block partials repeat exactly — LDS float atomics across the waves did not)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float* sb = smem;                      // [8][F][F]
  float* sdb0 = sb + NH * FF;            // [4][8][F][F]
  float* sg0 = sdb0 + 4 * NH * FF;       // [4][C]
  float* sgm = sg0 + 4 * C;              // [C] LN gamma (LDS reads do not queue behind the emission stores)
  float* rot = sgm + C;                  // [16][RS]
  float* sdb = sdb0 + wid * NH * FF;
  float* sg = sg0 + wid * C;
  const int lr = lane & 15, lg = lane >> 4;
  const int b = blockIdx.y;
  const int F4 = pad4(F), VW = T::PW * F4;
  constexpr int NVT = NV;
  const int R = NVT * 16;
  bf16* sq = reinterpret_cast<bf16*>(rot + 16 * RS) + wid * 4 * R * HS;
  bf16* sk = sq + R * HS;
  bf16* sv = sk + R * HS;
  bf16* sdo = sv + R * HS;
  // 16 zero rows past the last wave's slices (its last pixel's unmasked k-slot gathers read up to 12 rows into
  // them), then Li / D
  float* spad = reinterpret_cast<float*>(reinterpret_cast<bf16*>(rot + 16 * RS) + 4 * 4 * R * HS);
  float* sld = spad + 8 * HS + wid * 32;
  for (int e = tid; e < NH * FF; e += 256) sb[e] = bias[e] * LOG2E;
  for (int e = tid; e < 4 * NH * FF; e += 256) sdb0[e] = 0.f;
  for (int e = tid; e < 4 * C; e += 256) sg0[e] = 0.f;
  for (int e = tid; e < C; e += 256) sgm[e] = gamma[e];
  for (int e = tid; e < F * 32; e += 256) rot[(e >> 5) * RS + (e & 31)] = rotg[e];
  for (int e = tid; e < 8 * HS; e += 256) spad[e] = 0.f;
  __syncthreads();

  const int npg = (HW + T::PW - 1) / T::PW;
  const int nw = gridDim.x * 4;
  float dgam[DG_REG ? T::CT : 1][4];
#pragma unroll
  for (int ct = 0; ct < (DG_REG ? T::CT : 1); ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) dgam[ct][r] = 0.f;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  int fr[NV];
#pragma unroll
  for (int vt = 0; vt < NV; ++vt) fr[vt] = (vt * 16 + lr) % F4 < F ? (vt * 16 + lr) % F4 : 0;

  for (int pg = blockIdx.x * 4 + wid; pg < npg; pg += nw) {
    const int p0 = pg * T::PW;
    bf16x8 xf[T::NVTM][T::KS];
    tw_ln<C, NV>(x, sgm, nullptr, mr, xf, NVT, VW, F, F4, p0, HW, b, 0.f, lr, lg);
    int64_t vrow[T::NVTM];  // row of voxel (vt*16 + lane&15), -1 when outside the group
#pragma unroll
    for (int vt = 0; vt < T::NVTM; ++vt) {
      int64_t row = 0;
      vrow[vt] = tw_row(vt * 16 + lr, VW, F, F4, p0, HW, b, row) ? row : -1;
      if (vrow[vt] >= 0 && xn_out) {
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) stnt16(xn_out + row * C + ks * 32 + lg * 8, xf[vt][ks]);
      }
    }
    f32x4 dxacc[T::CT][T::NVTM];
#pragma unroll
    for (int ct = 0; ct < T::CT; ++ct)
#pragma unroll
      for (int vt = 0; vt < T::NVTM; ++vt) dxacc[ct][vt] = z4;
    // dy fragments of the wave's voxels, loaded once (not once per head)
    constexpr bool DYREG = C <= 64;
    bf16x8 dyr[DYREG ? T::NVTM : 1][DYREG ? T::KS : 1];
    if constexpr (DYREG) {
#pragma unroll
      for (int vt = 0; vt < T::NVTM; ++vt)
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks)  // unconditional load (row 0 when outside), then select
          dyr[vt][ks] = sel8(vrow[vt] >= 0, ldnt16(dy + (vrow[vt] >= 0 ? vrow[vt] : 0) * C + ks * 32 + lg * 8));
    }

    for (int h = 0; h < NH; ++h) {
      // issued ahead of the q/k/v GEMMs so its latency hides behind them: this head's log-sum-exp
      // of the wave's pixels (one per frame row lr)
      constexpr bool LPF = C <= 64;  // at C = 128 the 2 extra registers cost spills
      float Lp[T::PW];
#pragma unroll
      for (int pp = 0; pp < T::PW; ++pp) {
        if constexpr (LPF) {
          const bool ok = lr < F && p0 + pp < HW;
          const float v = lse[(((int64_t)b * NH + h) * HW + (ok ? p0 + pp : 0)) * F + (ok ? lr : 0)];
          Lp[pp] = ok ? v : 0.f;
        } else {
          Lp[pp] = 0.f;
        }
      }
      tw_qkv<C, NV>(wqkv, xf, h, fr, scale, rot, sq, sk, sv, lr, lg);
      // dO_h^T = W_out[:, h]^T . dy^T
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        bf16x8 a[T::KS];
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) a[ks] = ld_img(wout_t, h * 2 + dt, T::KS, ks, lane);  // image of W_out^T
#pragma unroll
        for (int vt = 0; vt < T::NVTM; ++vt) {
          if (vt < NVT) {
            f32x4 acc = z4;
#pragma unroll
            for (int ks = 0; ks < T::KS; ++ks) {
              bf16x8 dyf;
              if constexpr (DYREG) dyf = dyr[vt][ks];
              else dyf = sel8(vrow[vt] >= 0, ld16(dy + (vrow[vt] >= 0 ? vrow[vt] : 0) * C + ks * 32 + lg * 8));
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], dyf, acc, 0, 0, 0);
            }
            float o4[4] = {acc[0], acc[1], acc[2], acc[3]};
            store4(sdo + hs_off<R>(vt * 16 + lr, dt * 16 + lg * 4), o4);
          }
        }
      }
      // biases (log2 units): transposed entries (i = lr, j = 4g + r) and row-major (i = 4g + r, j = lr)
      float bt[4], brm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = lg * 4 + r;
        const bool ok = c < F && lr < F;
        bt[r] = ok ? sb[(h * F + lr) * F + c] : 0.f;
        brm[r] = ok ? sb[(h * F + c) * F + lr] : 0.f;
      }
      wave_lds_sync();
      // core backward per pixel; dq/dk/dv overwrite the pixel's own q/k/v rows at the end
      float dbr[4] = {0.f, 0.f, 0.f, 0.f};
      for (int pp = 0; pp < T::PW; ++pp) {
        const int p = p0 + pp;
        if (p >= HW) break;
        const int rb = pp * F4;
        float Li = Lp[0];
        if constexpr (LPF) {
#pragma unroll
          for (int q = 1; q < T::PW; ++q) Li = pp == q ? Lp[q] : Li;
        } else {
          const float v = lse[(((int64_t)b * NH + h) * HW + p) * F + (lr < F ? lr : 0)];
          Li = lr < F ? v : 0.f;
        }
        const int rr = rg_at(rb, hs_off<R>(lr < F ? lr : 0, lg * 8));  // rows past F read the pixel's row 0 (finite); every product is masked by ok / pt = 0
        const bf16x8 kr = ld16(sk + rr);
        const bf16x8 qr = ld16(sq + rr);
        const bf16x8 vr = ld16(sv + rr);
        const bf16x8 dor = ld16(sdo + rr);
        // -- transposed orientation: lane (g, i): entries (j = 4g + r, i)
        float D = 0.f;
        bf16x8 dst_b = zero8(), pt_b = zero8();
        {
          const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr, qr, z4, 0, 0, 0);    // S^T[j][i]
          const f32x4 dpt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vr, dor, z4, 0, 0, 0);  // dP^T[j][i]
          float pt[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = lg * 4 + r;
            const bool ok = j < F && lr < F;
            pt[r] = ok ? __builtin_amdgcn_exp2f(fmaf(st[r], LOG2E, bt[r]) - Li) : 0.f;
            D = fmaf(pt[r], dpt[r], D);
          }
          D = grp4_sum(D);
          if (lg == 0) { sld[lr] = Li; sld[16 + lr] = D; }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float ds = pt[r] * (dpt[r] - D);
            dbr[r] += ds;
            dst_b[r] = (bf16)ds;
            pt_b[r] = (bf16)pt[r];
          }
        }
        // k-slot gathers: slot (g, e<4) <-> frame 4g+e, column d = half*16 + (lane & 15)
        f32x4 dqt[2];
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          // (the 16x16x16 form used in tw_fwd / twh_bwd measured 4-6 % slower in this kernel: kept at K = 32)
          const bf16x8 kg = kslot_gather_raw<R>(sk, rb, half * 16, lane);  // dS^T / P^T are 0 at frames >= F
          const bf16x8 vg = kslot_gather_raw<R>(sv, rb, half * 16, lane);
          dqt[half] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kg, dst_b, z4, 0, 0, 0);  // dQ'^T[d][i]
          if (!o_out) continue;  // O written by the forward (cesm_tblock_fwd o)
          const f32x4 ot = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vg, pt_b, z4, 0, 0, 0);  // O^T[d][i]
          if (lr < F) {
            float oo[4] = {ot[0], ot[1], ot[2], ot[3]};
            stnt4(o_out + (((int64_t)b * F + lr) * HW + p) * INNER + h * DH + half * 16 + lg * 4, oo);
          }
        }
        // -- row-major orientation: lane (g, j): entries (i = 4g + r, j); L_i, D_i from lane i
        bf16x8 ds_b = zero8(), p_b = zero8();
        {
          const f32x4 s_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qr, kr, z4, 0, 0, 0);    // S[i][j]
          const f32x4 dp_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dor, vr, z4, 0, 0, 0);  // dP[i][j]
          wave_lds_sync();
          const f32x4 L4 = *reinterpret_cast<const f32x4*>(sld + lg * 4);
          const f32x4 D4 = *reinterpret_cast<const f32x4*>(sld + 16 + lg * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = lg * 4 + r;
            const float Lr = L4[r], Dr = D4[r];
            const bool ok = i < F && lr < F;
            const float pv = ok ? __builtin_amdgcn_exp2f(fmaf(s_[r], LOG2E, brm[r]) - Lr) : 0.f;
            p_b[r] = (bf16)pv;
            ds_b[r] = (bf16)(ok ? pv * (dp_[r] - Dr) : 0.f);
          }
        }
        f32x4 dkt[2], dvt[2];
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const bf16x8 qg = kslot_gather_raw<R>(sq, rb, half * 16, lane);
          const bf16x8 dog = kslot_gather_raw<R>(sdo, rb, half * 16, lane);
          dkt[half] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qg, ds_b, z4, 0, 0, 0);   // dK'^T[d][j]
          dvt[half] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dog, p_b, z4, 0, 0, 0);   // dV^T[d][j]
        }
        wave_lds_sync();  // all reads of this pixel's rows done before they are overwritten
        if (lr < F) {
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int d0 = half * 16 + lg * 4;
            float q4[4] = {dqt[half][0], dqt[half][1], dqt[half][2], dqt[half][3]};
            float k4[4] = {dkt[half][0], dkt[half][1], dkt[half][2], dkt[half][3]};
            float v4[4] = {dvt[half][0], dvt[half][1], dvt[half][2], dvt[half][3]};
            rope4(q4, rot, lr, d0, -1.f);  // dq = scale R^T dQ', dk = R^T dK' (frame lr)
            rope4(k4, rot, lr, d0, -1.f);
#pragma unroll
            for (int r = 0; r < 4; ++r) q4[r] *= scale;
            store4(sq + rg_at(rb, hs_off<R>(lr, d0)), q4);
            store4(sk + rg_at(rb, hs_off<R>(lr, d0)), k4);
            store4(sv + rg_at(rb, hs_off<R>(lr, d0)), v4);
          }
        }
        wave_lds_sync();
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (lr < F && lg * 4 + r < F) sdb[(h * F + lr) * F + lg * 4 + r] += dbr[r];
      wave_lds_sync();
      // dxn^T += W_qkv[h rows]^T . [dq|dk|dv]_h^T ; emit dqkv_h
#pragma unroll
      for (int kind = 0; kind < 3; ++kind) {
        const bf16* src = kind == 0 ? sq : (kind == 1 ? sk : sv);
        bf16x8 bf[T::NVTM];
#pragma unroll
        for (int vt = 0; vt < T::NVTM; ++vt) bf[vt] = vt < NVT ? ld16(src + hs_off<R>(vt * 16 + lr, lg * 8)) : zero8();
#pragma unroll
        for (int ct = 0; ct < T::CT; ++ct) {
          const bf16x8 a = ld_img(wqkv_t, ct, QKV / 32, kind * 8 + h, lane);  // image of W_qkv^T [C][768]
#pragma unroll
          for (int vt = 0; vt < T::NVTM; ++vt)
            if (vt < NVT) dxacc[ct][vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bf[vt], dxacc[ct][vt], 0, 0, 0);
        }
      }
      // emission after all of the head's weight loads: a load issued behind a store waits for it
      // (vmcnt counts both in issue order), so storing between the kinds stalled the next kind's W^T loads
      if (dqkv_out) {
#pragma unroll
        for (int kind = 0; kind < 3; ++kind) {
          const bf16* src = kind == 0 ? sq : (kind == 1 ? sk : sv);
#pragma unroll
          for (int vt = 0; vt < T::NVTM; ++vt) {
            if (vt >= NVT) break;
            int64_t row = 0;
            if (tw_row(vt * 16 + lr, VW, F, F4, p0, HW, b, row))
              stnt16(dqkv_out + row * QKV + kind * INNER + h * DH + lg * 8, ld16(src + hs_off<R>(vt * 16 + lr, lg * 8)));
          }
        }
      }
      wave_lds_sync();
    }
    // LN backward: dx = rstd*(g - mean(g) - xhat*mean(g*xhat)) + dy, g = dxn*gamma
    if ((int64_t)F * HW * C * 2 < 0x7fff0000) {  // uniform
      // every x / dy / stats load before the first dx store, the stores branch-free through a buffer resource over
      // sample b (rows outside the group go to an out-of-range offset, which the hardware drops): vmcnt retires in
      // issue order, so a load behind a store waits for it (the per-tile dy load -> dx store rounds)
      const int64_t s0 = (int64_t)b * F * HW;
      const __amdgpu_buffer_rsrc_t drs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(dx + s0 * C), (short)0, (int)((int64_t)F * HW * C * 2), 0x00020000);
      bf16x4 xr[T::NVTM][T::CT], dr[T::NVTM][T::CT];
      float2 mrv[T::NVTM];
      int voff[T::NVTM];
      bool okv[T::NVTM];
#pragma unroll
      for (int vt = 0; vt < T::NVTM; ++vt) {
        if (vt >= NVT) break;
        int64_t row = 0;
        okv[vt] = tw_row(vt * 16 + lr, VW, F, F4, p0, HW, b, row);
        row = okv[vt] ? row : 0;
        voff[vt] = okv[vt] ? (int)((row - s0) * C * 2) : 0x7fff8000;  // + co * 2 stays < INT_MAX, > num_records
        mrv[vt] = *reinterpret_cast<const float2*>(mr + row * 2);
#pragma unroll
        for (int ct = 0; ct < T::CT; ++ct) {
          xr[vt][ct] = __builtin_nontemporal_load(reinterpret_cast<const bf16x4*>(x + row * C + ct * 16 + lg * 4));
          dr[vt][ct] = __builtin_nontemporal_load(reinterpret_cast<const bf16x4*>(dy + row * C + ct * 16 + lg * 4));
        }
      }
#pragma unroll
      for (int vt = 0; vt < T::NVTM; ++vt) {
        if (vt >= NVT) break;
        const bool ok = okv[vt];
        const float mean = ok ? mrv[vt].x : 0.f, rstd = ok ? mrv[vt].y : 0.f;
        float s1 = 0.f, s2 = 0.f;
        float xh[T::CT][4];
#pragma unroll
        for (int ct = 0; ct < T::CT; ++ct) {
          const int co = ct * 16 + lg * 4;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            xh[ct][r] = ok ? ((float)xr[vt][ct][r] - mean) * rstd : 0.f;
            const float g = dxacc[ct][vt][r] * sgm[co + r];
            s1 += g;
            s2 = fmaf(g, xh[ct][r], s2);
            if constexpr (DG_REG) dgam[ct][r] = fmaf(dxacc[ct][vt][r], xh[ct][r], dgam[ct][r]);
          }
        }
        s1 = grp4_sum(s1);
        s2 = grp4_sum(s2);
        s1 /= C;
        s2 /= C;
#pragma unroll
        for (int ct = 0; ct < T::CT; ++ct) {
          const int co = ct * 16 + lg * 4;
          if constexpr (!DG_REG) {
            float d4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              d4[r] = dxacc[ct][vt][r] * xh[ct][r];
#pragma unroll
              for (int o = 1; o < 16; o <<= 1) d4[r] += __shfl_xor(d4[r], o, 64);
            }
            if (lr == 0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) sg[co + r] += d4[r];
            }
          }
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            o[r] = (bf16)(rstd * (dxacc[ct][vt][r] * sgm[co + r] - s1 - xh[ct][r] * s2) + (float)dr[vt][ct][r]);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(tw_u32x2, o), drs, voff[vt] + co * 2, 0, 0);
        }
      }
    } else
#pragma unroll
    for (int vt = 0; vt < T::NVTM; ++vt) {
      if (vt >= NVT) break;
      int64_t row = 0;
      const bool ok = tw_row(vt * 16 + lr, VW, F, F4, p0, HW, b, row);
      row = ok ? row : 0;  // loads unpredicated (row 0 outside the group), results selected
      const float m0 = mr[row * 2], r0 = mr[row * 2 + 1];
      const float mean = ok ? m0 : 0.f, rstd = ok ? r0 : 0.f;
      float s1 = 0.f, s2 = 0.f;
      float xh[T::CT][4];
#pragma unroll
      for (int ct = 0; ct < T::CT; ++ct) {
        const int co = ct * 16 + lg * 4;
        float xv[4];
        ldnt4(x + row * C + co, xv);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xh[ct][r] = ok ? (xv[r] - mean) * rstd : 0.f;
          const float g = dxacc[ct][vt][r] * sgm[co + r];
          s1 += g;
          s2 = fmaf(g, xh[ct][r], s2);
          if constexpr (DG_REG) dgam[ct][r] = fmaf(dxacc[ct][vt][r], xh[ct][r], dgam[ct][r]);
        }
      }
      s1 = grp4_sum(s1);
      s2 = grp4_sum(s2);
      s1 /= C;
      s2 /= C;
#pragma unroll
      for (int ct = 0; ct < T::CT; ++ct) {
        const int co = ct * 16 + lg * 4;
        if constexpr (!DG_REG) {
          float d4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            d4[r] = dxacc[ct][vt][r] * xh[ct][r];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) d4[r] += __shfl_xor(d4[r], o, 64);
          }
          if (lr == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) sg[co + r] += d4[r];
          }
        }
        float dv[4];
        ldnt4(dy + row * C + co, dv);
        if (ok) {
          float o4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o4[r] = rstd * (dxacc[ct][vt][r] * sgm[co + r] - s1 - xh[ct][r] * s2) + dv[r];
          stnt4(dx + row * C + co, o4);
        }
      }
    }
  }
  if constexpr (DG_REG) {
#pragma unroll
    for (int ct = 0; ct < T::CT; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = dgam[ct][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
        if (lr == 0) sg[ct * 16 + lg * 4 + r] += v;
      }
  }
  __syncthreads();
  const int S = NH * FF;
  for (int e = tid; e < S; e += 256) {
    const int h = e / FF, r = e - h * FF;
    dbias_part[(((int64_t)b * NH + h) * gridDim.x + blockIdx.x) * FF + r] =
        ((sdb0[e] + sdb0[S + e]) + sdb0[2 * S + e]) + sdb0[3 * S + e];
  }
  for (int e = tid; e < C; e += 256)
    dgamma_part[((int64_t)b * gridDim.x + blockIdx.x) * C + e] = ((sg0[e] + sg0[C + e]) + sg0[2 * C + e]) + sg0[3 * C + e];
}

__global__ void tb_sum_rows_kernel(const float* __restrict__ part, float* __restrict__ dst, int nrows, int C,
                                   int accumulate) {
  const int c = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < nrows; k += 64) s += part[(int64_t)k * C + c];
  s = wave_sum(s);
  if (threadIdx.x == 0) dst[c] = accumulate ? dst[c] + s : s;
}

template <int C>
static size_t tw_fwd_smem(int F) {  // NOLINT
  const int R = ((TW<C>::PW * F + 15) / 16) * 16;
  return (size_t)(((NH * F * F + 3) & ~3) + 16 * RS) * 4 + (size_t)4 * 3 * R * HS * 2 + 1024;  // + 16-row tail pad: k-slot gathers read up to 12 rows past the last slice
}
template <int C>
static size_t tw_bwd_smem(int F) {
  const int R = ((TW<C>::PW * F + 15) / 16) * 16;
  return (size_t)(5 * NH * F * F + 5 * C + 16 * RS) * 4 + (size_t)4 * 4 * R * HS * 2 + 8 * HS * 4 + 4 * 32 * 4;
}
template <typename K>
static void allow_smem(K kernel, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <int C, int NV, bool FOLD = false>
static void tw_fwd_launch_nv(const void* x, const float* gamma, const void* wqkv, const void* wout, const float* bias,
                             const float* rot, void* y, float* mr, float* lse, void* o, int B, int F, int HW,
                             float scale, float eps, hipStream_t stream) {
  const int npg = (int)cdiv(HW, TW<C>::PW);
  dim3 grid((unsigned)cdiv(npg, 4), B);
  const size_t sm = tw_fwd_smem<C>(F);
  allow_smem(tw_fwd_kernel<C, NV, FOLD>, sm);
  tw_fwd_kernel<C, NV, FOLD><<<grid, 256, sm, stream>>>((const bf16*)x, gamma, (const bf16*)wqkv, (const bf16*)wout,
                                                        bias, rot, (bf16*)y, mr, lse, (bf16*)o, F, HW, scale, eps);
}

template <int C>
static int tw_fwd_launch(const void* x, const float* gamma, const void* wqkv, const void* wout, const float* bias,
                         const float* rot, void* y, float* mr, float* lse, void* o, int B, int F, int HW, float scale,
                         float eps, hipStream_t stream) {
  const int nv = (TW<C>::PW * F + 15) / 16;
  switch (nv) {
    case 1: tw_fwd_launch_nv<C, 1>(x, gamma, wqkv, wout, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream); break;
    case 2:
      if constexpr (TW<C>::PW >= 2) { tw_fwd_launch_nv<C, 2>(x, gamma, wqkv, wout, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream); break; }
      return CESM_EUNSUPPORTED;
    case 3:
      if constexpr (TW<C>::PW >= 3) { tw_fwd_launch_nv<C, 3>(x, gamma, wqkv, wout, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream); break; }
      return CESM_EUNSUPPORTED;
    case 4:
      if constexpr (TW<C>::PW >= 4) { tw_fwd_launch_nv<C, 4>(x, gamma, wqkv, wout, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream); break; }
      return CESM_EUNSUPPORTED;
    default:
      return CESM_EUNSUPPORTED;
  }
  return cesm_launch_status();
}

template <int C, int NV>
static void tw_bwd_launch_nv(const void* x, const void* dy, const float* gamma, const float* mr, const float* lse,
                             const void* wqkv, const void* wqkv_t, const void* wout_t, const float* bias,
                             const float* rot, void* dx, void* dqkv, void* o, void* xn, float* dbias_part,
                             float* dgamma_part, dim3 grid, int F, int HW, float scale, hipStream_t stream) {
  const size_t sm = tw_bwd_smem<C>(F);
  allow_smem(tw_bwd_kernel<C, NV>, sm);
  tw_bwd_kernel<C, NV><<<grid, 256, sm, stream>>>((const bf16*)x, (const bf16*)dy, gamma, mr, lse, (const bf16*)wqkv,
                                                  (const bf16*)wqkv_t, (const bf16*)wout_t, bias, rot, (bf16*)dx,
                                                  (bf16*)dqkv, (bf16*)o, (bf16*)xn, dbias_part, dgamma_part, F, HW,
                                                  scale);
}

template <int C>
static int tw_bwd_launch(const void* x, const void* dy, const float* gamma, const float* mr, const float* lse,
                         const void* wqkv, const void* wqkv_t, const void* wout_t, const float* bias, const float* rot,
                         void* dx, void* dqkv, void* o, void* xn, float* dbias_part, float* dgamma_part, dim3 grid,
                         int F, int HW, float scale, hipStream_t stream) {
  const int nv = (TW<C>::PW * F + 15) / 16;
#define TWB_ARGS x, dy, gamma, mr, lse, wqkv, wqkv_t, wout_t, bias, rot, dx, dqkv, o, xn, dbias_part, dgamma_part, grid, F, HW, scale, stream
  switch (nv) {
    case 1: tw_bwd_launch_nv<C, 1>(TWB_ARGS); break;
    case 2:
      if constexpr (TW<C>::PW >= 2) { tw_bwd_launch_nv<C, 2>(TWB_ARGS); break; }
      return CESM_EUNSUPPORTED;
    case 3:
      if constexpr (TW<C>::PW >= 3) { tw_bwd_launch_nv<C, 3>(TWB_ARGS); break; }
      return CESM_EUNSUPPORTED;
    case 4:
      if constexpr (TW<C>::PW >= 4) { tw_bwd_launch_nv<C, 4>(TWB_ARGS); break; }
      return CESM_EUNSUPPORTED;
    default:
      return CESM_EUNSUPPORTED;
  }
#undef TWB_ARGS
  return CESM_OK;
}

}  // namespace

// ============================================================================================
// Head-parallel fused backward with in-kernel weight gradients (C = 64, 4*F <= 48).
//
// A block of 8 waves processes one pixel group (4 pixels x F frames) at a time, wave h owning head h:
// LN (block-cooperative, xhat and dy tiles in LDS) -> per wave: q/k/v_h and dO_h GEMMs, the attention-core
// backward, dxn_h = W'_h^T dqkv_h (partial over heads) and dW'_h += dqkv_h^T xhat (MFMA accumulators that
// stay in registers for the whole kernel) -> the 8 partial dxn summed through LDS -> LN backward -> dx.
// Nothing per voxel is written but dx: the 768-channel dqkv and xn tensors of the wave-private kernel
// (1.8 KB per voxel, re-read by the weight-gradient GEMM) do not exist on this path.
// gamma is folded into the weights: W' = W diag(gamma) (images built from the fp32 master weight), so the
// GEMMs take xhat and the dxn GEMM yields g = gamma * dxn directly; the weight gradient leaves the kernel
// as dW' = sum dqkv^T xhat, and twh_dw_finalize turns it into dW = dW' diag(gamma) and
// dgamma_c = sum_j W[j][c] dW'[j][c] (the LN gamma gradient sum_v dxn*xhat, regrouped).
// ============================================================================================
// round-2 helpers of twh_bwd (80-B slice rows, see the TWH section)
__device__ __forceinline__ bf16x8 kslot_gather_hld(const bf16* tile, int rb, int c0, int F, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + (rb + 4 * g + q) * HLD + c0 + 4 * p));
  bf16x8 r = zero8();
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (4 * g + e < F) r[e] = __builtin_bit_cast(bf16, (short)v[e]);
  return r;
}
__device__ __forceinline__ bf16x8 kslot_gather_ld(const bf16* tile, int ld, int rb, int c0, int F, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + (rb + 4 * g + q) * ld + c0 + 4 * p));
  bf16x8 r = zero8();
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (4 * g + e < F) r[e] = __builtin_bit_cast(bf16, (short)v[e]);
  return r;
}
// Unmasked k-slot gathers (round 3): where the other MFMA operand is exactly zero at every k-slot of a frame >= F
// (P, dS and their transposes are 0 there), the rows read past the pixel's F frames -- the next pixel's finite
// rows, or the zero-initialised tail pad past the last slice -- contribute 0, so the 4 per-element selects
// (v_cndmask + repacking, ~15 % of twh_bwd's VALU) are not needed
__device__ __forceinline__ s16x4 kslot4_hld(const bf16* tile, int rb, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + (rb + 4 * g + q) * HLD + c0 + 4 * p));
}
__device__ __forceinline__ s16x4 kslot4_ld(const bf16* tile, int ld, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + (4 * g + q) * ld + 4 * p));
}

// twh_bwd: pixels whose attention-core backward is interleaved phase by phase.  Fixed at 1 (round 2: 3375 vs
// 3460 us with 2, 2 spills vs 10); 2 no longer fits the LDS next to the round-3 tiles, so it is not a knob.
constexpr int TWH_PG = 1;
// The dxn GEMM's W'^T fragments in a ring of this depth (round 2: 3 +3-4 %, no ring +4.5 %).
constexpr int TWH_RING = 2;
// Measured and removed (A/B records: profiles/r2_v13_*, r3_attn_knobs_ab.txt, r4_attn_variants_ab.txt, r5_prio_ab.txt,
// r5_dxt_tb.txt, r5f_prefetch_pos_tb.txt, r5f_twh_dx_late_tb.txt, r5f_twh_ldq_early_tb.txt, r5_twh_dwout_env_ab.txt):
// q/k/v weights without the double-buffered batches (+1.5-2 %), the dO weights loaded after the q/k/v batches
// (+1-2.5 %), scalar instead of packed fp32 in the softmax-gradient step (+0.5 %), the next group's x / dy prefetch
// after the head phase (neutral), the dx stores right after LN backward or after the first weight batch (+0.8 %),
// s_setprio for waves 4-7 (neutral), dxn by whole output tiles after a block barrier (3.82 -> 4.35 ms per call), and the
// to_out weight gradient in-kernel (DWO: 32 persistent accumulators, 58-93 spilled registers, 3.3 -> 5.3 ms per call
// -- more than the forward's O write and the O^T dy GEMM it removes).
constexpr int TH_XLD = 72;   // xhat / dy tile row stride (bf16, 144-B rows)
constexpr int TH_NVMAX = 3;  // voxel tiles per group (4*F <= 48): the 8 slices then fit in LDS
// twh_bwd keeps round 2's padded tiles (80-B slice rows, 144-B xhat / dy rows, 68-float partial rows): the region
// layouts of the other fused kernels remove its LDS bank conflicts too, but their per-site lane offsets push this
// 256-VGPR kernel into spills or, recomputed per group, into +7 % VALU -- 4.27-4.50 vs 4.06-4.08 ms per call at the
// level-0 size (profiles/r3_lds_layout_ab.txt); its limiter is VALU issue, not LDS
constexpr int TWH_PLD = 68;  // fp32 row stride of a wave's partial dxn rows (written over its own slices)

// per-wave slice region: q | k | v | dO [R][HLD] + a 16-row zero pad: the unmasked k-slot gathers of the wave's last
// pixel read up to (PW-1)F + 16 - R <= 12 rows past dO (F = 4), which must be finite (the next wave's region may
// still hold fp32 partial rows)
#define TWH_WSTRIDE(R) (4 * (R) * HLD + 16 * HLD)
static size_t twh_smem(int F, int NV) {
  (void)F;
  const int R = NV * 16;
  return (size_t)16 * RS * 4 + (size_t)8 * TWH_PG * 2 * 256 * 2 + (size_t)(2 * R) * TH_XLD * 2 +
         (size_t)8 * TWH_WSTRIDE(R) * 2;
}

template <int NV>
__global__ __launch_bounds__(512, 1) void twh_bwd_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, const float* __restrict__ mr,
    const float* __restrict__ lse, const bf16* __restrict__ wqkv, const bf16* __restrict__ wqkv_t,
    const bf16* __restrict__ wout_t, const float* __restrict__ bias, const float* __restrict__ rotg,
    bf16* __restrict__ dx, bf16* __restrict__ o_out, float* __restrict__ dw_slab, float* __restrict__ dbias_part,
    int B, int F, int HW, float scale) {
  constexpr int C = 64;
  using T = TW<C, NV>;
  constexpr int R = NV * 16;
  static_assert(TWH_PLD * 4 <= 4 * HLD * 2, "partial dxn rows fit over the wave's slices");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int FF = F * F;
  float* rot = smem;                                 // [16][RS]
  float* trbuf = rot + 16 * RS;                      // [8 waves][TWH_PG][2][16][16] bf16 P / dS tiles
  bf16* xt = reinterpret_cast<bf16*>(trbuf) + 8 * TWH_PG * 2 * 256;  // [R][TH_XLD] xhat (bf16)
  bf16* dyt = xt + R * TH_XLD;                       // [R][TH_XLD] dy
  bf16* slices = dyt + R * TH_XLD;                   // 8 x [q|k|v|dO][R][HLD]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int h = wid;
  bf16* sq = slices + wid * TWH_WSTRIDE(R);
  bf16* sk = sq + R * HLD;
  bf16* sv = sk + R * HLD;
  bf16* sdo = sv + R * HLD;
  for (int e = tid; e < F * 32; e += 512) rot[(e >> 5) * RS + (e & 31)] = rotg[e];
  // the wave's 16-row pad past dO (never written afterwards: the partial rows fit over the slices)
  for (int e = lane; e < 8 * HLD; e += 64) reinterpret_cast<float*>(sq + 4 * R * HLD)[e] = 0.f;
  // this wave's (head's) bias entries, log2 units: transposed (i = lr, j = 4g + r) and row-major (i = 4g + r, j = lr)
  float bt[4], brm[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = lg * 4 + r;
    const bool ok = c < F && lr < F;
    const int i0 = ok ? lr : 0, c0 = ok ? c : 0;
    const float b0 = bias[(h * F + i0) * F + c0], b1 = bias[(h * F + c0) * F + i0];
    bt[r] = ok ? b0 * LOG2E : 0.f;
    brm[r] = ok ? b1 * LOG2E : 0.f;
  }

  const int VW = T::PW * F;
  const int npg = (HW + T::PW - 1) / T::PW;
  const int ngroups = B * npg;
  // LN / LN-backward role of this thread: voxel vv of the group, channels 8cc..8cc+7
  const int vv = tid >> 3, cc = tid & 7;
  int fr[NV];
#pragma unroll
  for (int vt = 0; vt < NV; ++vt) fr[vt] = (vt * 16 + lr) % F;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};

  // the voxel row of (group gg, voxel v) or -1
  auto vrow = [&](int gg, int v) -> int64_t {
    const int b = gg / npg, pg = gg - b * npg;
    if (v >= VW) return -1;
    const int pp = v / F, f = v - pp * F, p = pg * T::PW + pp;
    if (p >= HW) return -1;
    return ((int64_t)b * F + f) * HW + p;
  };
  // prefetch registers: x, dy chunk and (mean, rstd) of this thread's voxel in the next group
  bf16x8 xpf = zero8(), dpf = zero8();
  float mpf = 0.f, rpf = 0.f;
  bool okpf = false;
  auto prefetch = [&](int gg) {
    const int64_t row = gg < ngroups && vv < R ? vrow(gg, vv) : -1;
    okpf = row >= 0;
    const int64_t rr = okpf ? row : 0;  // unconditional loads, selected afterwards
    xpf = ldnt16(x + rr * C + cc * 8);
    dpf = ldnt16(dy + rr * C + cc * 8);
    mpf = mr[rr * 2];
    rpf = mr[rr * 2 + 1];
  };

  // weight-gradient accumulators dW'_h [q|k|v x 32 rows][64]: 6 row tiles x 4 column tiles
  f32x4 dwacc[6][4];
#pragma unroll
  for (int m = 0; m < 6; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) dwacc[m][n] = z4;
  float dbacc[4] = {0.f, 0.f, 0.f, 0.f};

  prefetch(blockIdx.x);
  // the previous group's dx chunk of this thread and its row (-1: none): stored after this group's q/k/v/dO weight
  // loads (vmcnt counts loads and stores in issue order: stored before them, the loads' first wait also waited for
  // the stores; round 5 -0.8 %)
  bf16x8 dx_pend = zero8();
  int64_t dx_row = -1;
  for (int gg = blockIdx.x; gg < ngroups; gg += gridDim.x) {
    const int b = gg / npg, p0 = (gg - b * npg) * T::PW;
    // ---- LN of the group (this thread's voxel chunk) from the prefetch registers
    float rstd_cur = 0.f;
    if (vv < R) {
      const bool ok = okpf;
      bf16x8 xh, dv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[e] = (bf16)(ok ? ((float)xpf[e] - mpf) * rpf : 0.f);
        dv[e] = ok ? dpf[e] : (bf16)0.f;
      }
      *reinterpret_cast<bf16x8*>(xt + vv * TH_XLD + cc * 8) = xh;
      *reinterpret_cast<bf16x8*>(dyt + vv * TH_XLD + cc * 8) = dv;
      rstd_cur = ok ? rpf : 0.f;
    }
    const bool ok_cur = okpf;
    const int oz = opaque_zero();
    const bf16* wq_g = wqkv + oz;
    const bf16* wqt_g = wqkv_t + oz;
    const bf16* wot_g = wout_t + oz;
    // q/k/v weight fragments in two-tile batches, double-buffered: batch 0 issued before barrier A (its L2
    // latency overlaps the barrier wait), batch c+1 issued before batch c's MFMAs; the dO GEMM's weights during the
    // last batch
    constexpr int QB = 2;
    bf16x8 wqa[2][QB][T::KS];
    bf16x8 wob[2][T::KS];
    auto ldq = [&](int c0, int buf) {
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        const int ct = c0 + u, mt = (ct >> 1) * 16 + h * 2 + (ct & 1);
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) wqa[buf][u][ks] = ld_img(wq_g, mt, T::KS, ks, lane);
      }
    };
    ldq(0, 0);
    __syncthreads();  // (A) tiles of this group ready; previous group's partials consumed
    prefetch(gg + gridDim.x);  // next group's x / dy / stats: in flight during the head phase

    // ---- head phase: wave h
    float Lp[T::PW];
#pragma unroll
    for (int pp = 0; pp < T::PW; ++pp) {
      const bool ok = lr < F && p0 + pp < HW;
      const float v = lse[(((int64_t)b * NH + h) * HW + (ok ? p0 + pp : 0)) * F + (ok ? lr : 0)];
      Lp[pp] = ok ? v : 0.f;
    }
    {
      bf16x8 xf[NV][T::KS];
#pragma unroll
      for (int vt = 0; vt < NV; ++vt)
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) xf[vt][ks] = ld16(xt + (vt * 16 + lr) * TH_XLD + ks * 32 + lg * 8);
#pragma unroll
      for (int c0 = 0; c0 < 6; c0 += QB) {
        const int buf = (c0 / QB) & 1;
        if (c0 + QB < 6) ldq(c0 + QB, buf ^ 1);
        else {  // the dO GEMM's W_out^T fragments, in flight during the last q/k/v batch
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int ks = 0; ks < T::KS; ++ks) wob[dt][ks] = ld_img(wot_g, h * 2 + dt, T::KS, ks, lane);
        }
        // batched (round 4), one 16-dim half at a time: the half's RoPE coefficients read first, its NV tiles issued
        // back to back, then their epilogues (round 3: one MFMA -> s_nop -> LDS read -> wait -> VALU -> store chain
        // per tile; both halves at once spill at 256 VGPRs)
#pragma unroll
        for (int ub = 0; ub < QB; ++ub) {
          const int ct = c0 + ub, kind = ct >> 1, u = ct & 1;
          bf16* dst = kind == 0 ? sq : (kind == 1 ? sk : sv);
          f32x4 cs[NV];
          if (kind < 2) {
#pragma unroll
            for (int vt = 0; vt < NV; ++vt) cs[vt] = *reinterpret_cast<const f32x4*>(rot + fr[vt] * RS + u * 16 + lg * 4);
          }
          f32x4 qacc[NV];
#pragma unroll
          for (int vt = 0; vt < NV; ++vt) {
            qacc[vt] = z4;
#pragma unroll
            for (int ks = 0; ks < T::KS; ++ks)
              qacc[vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wqa[buf][ub][ks], xf[vt][ks], qacc[vt], 0, 0, 0);
          }
#pragma unroll
          for (int vt = 0; vt < NV; ++vt) {
            float o4[4] = {qacc[vt][0], qacc[vt][1], qacc[vt][2], qacc[vt][3]};  // q: scale in the weights
            if (kind < 2) rope4c(o4, cs[vt]);
            store4(dst + (vt * 16 + lr) * HLD + u * 16 + lg * 4, o4);
          }
        }
      }
    }
    // dO_h^T = W_out[:, h]^T . dy^T
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const auto& a = wob[dt];
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) {
        f32x4 acc = z4;
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], ld16(dyt + (vt * 16 + lr) * TH_XLD + ks * 32 + lg * 8),
                                                        acc, 0, 0, 0);
        float o4[4] = {acc[0], acc[1], acc[2], acc[3]};
        store4(sdo + (vt * 16 + lr) * HLD + dt * 16 + lg * 4, o4);
      }
    }
    if (dx_row >= 0) {  // the previous group's dx, behind this group's q/k/v/dO weight loads
      __builtin_amdgcn_sched_barrier(0);
      stnt16(dx + dx_row * C + cc * 8, dx_pend);
    }
    wave_lds_sync();
    // attention-core backward, TWH_PG pixels interleaved phase by phase; only the transposed orientation is
    // computed (S^T, dP^T on MFMA, softmax rows per lane), P and dS reach the row-major orientation of the
    // dK / dV products through a 16 x 16 bf16 LDS tile and the hardware transpose read
    constexpr int PG = TWH_PG;
    bf16* trt = reinterpret_cast<bf16*>(trbuf) + wid * PG * 2 * 256;  // [PG][P^T, dS^T][16][16]
    for (int pp0 = 0; pp0 < T::PW; pp0 += PG) {
      f32x4 st[PG], dpt[PG];
#pragma unroll
      for (int u = 0; u < PG; ++u) {
        const int rb = (pp0 + u) * F;
        const int rr = rb + (lr < F ? lr : 0);
        const bf16x8 kr = ld16(sk + rr * HLD + lg * 8);
        const bf16x8 qr = ld16(sq + rr * HLD + lg * 8);
        const bf16x8 vr = ld16(sv + rr * HLD + lg * 8);
        const bf16x8 dor = ld16(sdo + rr * HLD + lg * 8);
        st[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr, qr, z4, 0, 0, 0);    // S^T[j][i]
        dpt[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vr, dor, z4, 0, 0, 0);  // dP^T[j][i]
      }
      s16x4 dst_b[PG], pa_b[PG];
#pragma unroll
      for (int u = 0; u < PG; ++u) {
        const bool pix = p0 + pp0 + u < HW;
        float Li = Lp[0];
#pragma unroll
        for (int q = 1; q < T::PW; ++q) Li = pp0 + u == q ? Lp[q] : Li;
        float pt[4], D = 0.f;
        // two elements per VALU op (v_pk_fma / v_pk_add / v_pk_mul_f32) where the order allows, same results
        float ds4[4];
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f32x2 x2 = __builtin_elementwise_fma(f32x2{st[u][r], st[u][r + 1]}, f32x2{LOG2E, LOG2E},
                                                     f32x2{bt[r], bt[r + 1]}) - f32x2{Li, Li};
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const bool ok = pix && lg * 4 + r + e < F && lr < F;
            pt[r + e] = ok ? __builtin_amdgcn_exp2f(x2[e]) : 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) D = fmaf(pt[r], dpt[u][r], D);
        D = grp4_sum(D);
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f32x2 d2 = f32x2{pt[r], pt[r + 1]} * (f32x2{dpt[u][r], dpt[u][r + 1]} - f32x2{D, D});
          const f32x2 a2 = f32x2{dbacc[r], dbacc[r + 1]} + d2;
          dbacc[r] = a2[0];
          dbacc[r + 1] = a2[1];
          ds4[r] = d2[0];
          ds4[r + 1] = d2[1];
        }
        bf16x4 p4, d4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          d4[r] = (bf16)ds4[r];
          p4[r] = (bf16)pt[r];
        }
        dst_b[u] = __builtin_bit_cast(s16x4, d4);
        pa_b[u] = __builtin_bit_cast(s16x4, p4);
        // tile[i = lr][j = 4g .. 4g+3]
        *reinterpret_cast<bf16x4*>(trt + (u * 2 + 0) * 256 + lr * 16 + lg * 4) = p4;
        *reinterpret_cast<bf16x4*>(trt + (u * 2 + 1) * 256 + lr * 16 + lg * 4) = d4;
      }
      f32x4 dqt[PG][2];
#pragma unroll
      for (int u = 0; u < PG; ++u)
#pragma unroll
        for (int half = 0; half < 2; ++half)
          dqt[u][half] = mfma_k16(kslot4_hld(sk, (pp0 + u) * F, half * 16, lane), dst_b[u], z4);  // dQ'^T[d][i]
      wave_lds_sync();  // P / dS tiles visible
      f32x4 dkt[PG][2], dvt[PG][2];
#pragma unroll
      for (int u = 0; u < PG; ++u) {
        const s16x4 p_b = kslot4_ld(trt + (u * 2 + 0) * 256, 16, lane);   // P[i = 4g+e][j = lr]
        const s16x4 ds_b = kslot4_ld(trt + (u * 2 + 1) * 256, 16, lane);  // dS[i = 4g+e][j = lr]
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int rb = (pp0 + u) * F;
          dkt[u][half] = mfma_k16(kslot4_hld(sq, rb, half * 16, lane), ds_b, z4);   // dK'^T[d][j]
          dvt[u][half] = mfma_k16(kslot4_hld(sdo, rb, half * 16, lane), p_b, z4);   // dV^T[d][j]
        }
      }
      // O^T[d][i] = V^T . P^T of these pixels (o_out: the to_out weight gradient's input, round 6), stored straight
      // away (8 B per lane and half).  Parking it in the pixels' dead dO rows and storing it after the dW or the dxn
      // GEMM measured slower (3884-4325 vs 3696-3992 us per level-0 call: 23-45 more spilled registers,
      // profiles/r6g_twh_o_ab.txt); lane pairs exchanging halves by v_permlane16_swap for one 16-B store per lane
      // measured the same (+301 / +315 us for the emission, profiles/r6p_twh_o_paired_stores.txt)
      if (o_out) {  // uniform
#pragma unroll
        for (int u = 0; u < PG; ++u) {
          f32x4 ot[2];
#pragma unroll
          for (int half = 0; half < 2; ++half) ot[half] = mfma_k16(kslot4_hld(sv, (pp0 + u) * F, half * 16, lane), pa_b[u], z4);
          if (lr < F && p0 + pp0 + u < HW) {
            bf16* orow = o_out + (((int64_t)b * F + lr) * HW + p0 + pp0 + u) * INNER + h * DH + lg * 4;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
              bf16x4 o4;
#pragma unroll
              for (int r = 0; r < 4; ++r) o4[r] = (bf16)ot[half][r];
              __builtin_nontemporal_store(__builtin_bit_cast(uint64_t, o4), reinterpret_cast<uint64_t*>(orow + half * 16));
            }
          }
        }
      }
      wave_lds_sync();  // all reads of these pixels' rows (and the tiles) done before they are overwritten
#pragma unroll
      for (int u = 0; u < PG; ++u) {
        const int rb = (pp0 + u) * F;
        if (lr < F && p0 + pp0 + u < HW) {
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int d0 = half * 16 + lg * 4;
            float q4[4] = {dqt[u][half][0], dqt[u][half][1], dqt[u][half][2], dqt[u][half][3]};
            float k4[4] = {dkt[u][half][0], dkt[u][half][1], dkt[u][half][2], dkt[u][half][3]};
            float v4[4] = {dvt[u][half][0], dvt[u][half][1], dvt[u][half][2], dvt[u][half][3]};
            // dq~ = R^T dQ' (the gradient w.r.t. the scaled q rows the images hold: twh_dw_reduce applies the
            // scale to their weight gradient), dk = R^T dK'
            rope4(q4, rot, lr, d0, -1.f);
            rope4(k4, rot, lr, d0, -1.f);
            store4(sq + (rb + lr) * HLD + d0, q4);
            store4(sk + (rb + lr) * HLD + d0, k4);
            store4(sv + (rb + lr) * HLD + d0, v4);
          }
        }
      }
    }
    wave_lds_sync();
    {
      // the dxn GEMM's W'^T fragments (kind, ct) in a TWH_RING-deep ring: the first in flight during the dW GEMM
      bf16x8 wring[TWH_RING];
      auto ldw = [&](int idx) { return ld_img(wqt_g, idx % T::CT, QKV / 32, (idx / T::CT) * 8 + h, lane); };
  #pragma unroll
      for (int r = 0; r < TWH_RING - 1; ++r) wring[r] = ldw(r);
      // dW'_h += dqkv_h^T . xhat over the group's voxels (K = voxels, 16 per step; padded rows are zero)
  #pragma unroll
      for (int kk = 0; kk < NV; ++kk) {
        s16x4 bx[4];
  #pragma unroll
        for (int nt = 0; nt < 4; ++nt) bx[nt] = tr4(xt, TH_XLD, kk * 16, nt * 16, lane);
  #pragma unroll
        for (int m = 0; m < 6; ++m) {
          const bf16* src = (m >> 1) == 0 ? sq : ((m >> 1) == 1 ? sk : sv);
          const s16x4 a = tr4(src, HLD, kk * 16, (m & 1) * 16, lane);
  #pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            dwacc[m][nt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bx[nt], dwacc[m][nt], 0, 0, 0);
        }
      }
      // dxn'_h^T = W'_qkv[h rows]^T . dqkv_h^T (this head's share; gamma folded: the sum over heads is
      // g = gamma * dxn), kept in registers, then written as fp32 rows over the wave's own slices
      f32x4 dxacc[T::CT][NV];
  #pragma unroll
      for (int ct = 0; ct < T::CT; ++ct)
  #pragma unroll
        for (int vt = 0; vt < NV; ++vt) dxacc[ct][vt] = z4;
  #pragma unroll
      for (int kind = 0; kind < 3; ++kind) {
        const bf16* src = kind == 0 ? sq : (kind == 1 ? sk : sv);
  #pragma unroll
        for (int ct = 0; ct < T::CT; ++ct) {
          const int idx = kind * T::CT + ct;
          if (idx + TWH_RING - 1 < 3 * T::CT) wring[(idx + TWH_RING - 1) % TWH_RING] = ldw(idx + TWH_RING - 1);
          const bf16x8 a = wring[idx % TWH_RING];
  #pragma unroll
          for (int vt = 0; vt < NV; ++vt)
            dxacc[ct][vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ld16(src + (vt * 16 + lr) * HLD + lg * 8),
                                                                    dxacc[ct][vt], 0, 0, 0);
        }
      }
      wave_lds_sync();  // every read of this wave's slices done: they now take its partial dxn rows
      {
        float* part = reinterpret_cast<float*>(sq);
  #pragma unroll
        for (int ct = 0; ct < T::CT; ++ct)
  #pragma unroll
          for (int vt = 0; vt < NV; ++vt)
            *reinterpret_cast<f32x4*>(part + (vt * 16 + lr) * TWH_PLD + ct * 16 + lg * 4) = dxacc[ct][vt];
      }
      __syncthreads();  // (B) every head's partial written

      // ---- LN backward of this thread's voxel chunk: dx = rstd (g - mean(g) - xhat mean(g xhat)) + dy
      {
        const int v = vv < R ? vv : 0;
        float g[8];
  #pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = 0.f;
  #pragma unroll
        for (int w = 0; w < 8; ++w) {
          const float* pw = reinterpret_cast<const float*>(slices + w * TWH_WSTRIDE(R)) + v * TWH_PLD + cc * 8;
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(pw);
          const f32x4 a1 = *reinterpret_cast<const f32x4*>(pw + 4);
  #pragma unroll
          for (int e = 0; e < 4; ++e) { g[e] += a0[e]; g[4 + e] += a1[e]; }
        }
        const bf16x8 xh = *reinterpret_cast<const bf16x8*>(xt + v * TH_XLD + cc * 8);
        const bf16x8 dv = *reinterpret_cast<const bf16x8*>(dyt + v * TH_XLD + cc * 8);
        float s1 = 0.f, s2 = 0.f;
  #pragma unroll
        for (int e = 0; e < 8; ++e) { s1 += g[e]; s2 = fmaf(g[e], (float)xh[e], s2); }
  #pragma unroll
        for (int o = 1; o < 8; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
        s1 *= 1.f / C;
        s2 *= 1.f / C;
  #pragma unroll
        for (int e = 0; e < 8; ++e) dx_pend[e] = (bf16)(rstd_cur * (g[e] - s1 - (float)xh[e] * s2) + (float)dv[e]);
        dx_row = vv < R && ok_cur ? vrow(gg, vv) : -1;
      }
    }
  }
  if (dx_row >= 0) stnt16(dx + dx_row * C + cc * 8, dx_pend);
  // ---- per-block outputs: dW'_h rows of the slab, dbias partials (cesm_relpos_bwd layout, B = 1)
  float* slab = dw_slab + (int64_t)blockIdx.x * QKV * C;
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const int j0 = (m >> 1) * INNER + h * DH + (m & 1) * 16 + lg * 4;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(int64_t)(j0 + r) * C + nt * 16 + lr] = dwacc[m][nt][r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = lg * 4 + r;
    if (lr < F && j < F) dbias_part[((int64_t)h * gridDim.x + blockIdx.x) * FF + lr * F + j] = dbacc[r];
  }
}



extern "C" {

// Fused forward of Residual(PreNorm(temporal Attention)): x,y [B*F*HW][C] bf16 (channels-last),
// wqkv [768][C] / wout [C][256] packed bf16, bias [8][F][F], rot [F][16][2].
// mr [B*F*HW][2] (LN mean, rstd) and lse [B][8][HW][F] are saved for the backward (may be null).
int cesm_tblock_fwd(const void* x, const float* gamma, const void* wqkv, const void* wout, const float* bias,
                    const float* rot, void* y, float* mr, float* lse, void* o, void* wimg, int B, int F, int HW, int C,
                    float scale, float eps, hipStream_t stream) {
  if (F < 1 || F > 16) return CESM_EUNSUPPORTED;
  if (o && C > 256) return CESM_EUNSUPPORTED;  // only the wave-private kernels write O
  if (C <= 256) {  // the wave-private kernels read weight fragments from images (1-KiB lines)
    bf16* iq = (bf16*)wimg;
    bf16* io = iq + 768 * C;
    frag_image(wqkv, iq, 768, C, stream);
    frag_image(wout, io, C, INNER, stream);
    wqkv = iq;
    wout = io;
  }
  switch (C) {
    case 64: return tw_fwd_launch<64>(x, gamma, wqkv, wout, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream);
    case 128: return tw_fwd_launch<128>(x, gamma, wqkv, wout, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream);
    case 256: return tw_fwd_launch<256>(x, gamma, wqkv, wout, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream);
    case 512: {
      dim3 grid((unsigned)cdiv(HW, TB<512>::P), B);
      tblock_fwd_kernel<512><<<grid, 256, 0, stream>>>((const bf16*)x, gamma, (const bf16*)wqkv, (const bf16*)wout,
                                                       bias, rot, (bf16*)y, mr, lse, F, HW, scale, eps);
      break;
    }
    default:
      return CESM_EUNSUPPORTED;
  }
  return cesm_launch_status();
}

static int tb_bwd_P(int C) { return C >= 256 ? 1 : 256 / C; }

// blocks per sample used by cesm_tblock_bwd (grid-stride over pixel groups)
int cesm_tblock_bwd_nblk(int B, int F, int HW, int C) {
  (void)F;
  if (C <= 256) {
    const int pw = C <= 64 ? 4 : (C == 128 ? 2 : 1);
    const int nwg = (int)cdiv(cdiv(HW, pw), 4);  // 4 waves per block, one pixel group each
    const int target = std::max(1, 512 / std::max(B, 1));
    return std::min(nwg, target);
  }
  const int npg = (int)cdiv(HW, tb_bwd_P(C));
  const int target = std::max(1, 1024 / std::max(B, 1));
  return std::min(npg, target);
}

// Fused backward of the temporal-attention block (dx path). x, dy, dx [B*F*HW][C] bf16; gamma [C];
// mr, lse from cesm_tblock_fwd; wqkv [768][C], wqkv_t [C][768], wout_t [256][C] packed bf16.
// Emits (each may be null) dqkv [B*F*HW][768], o [B*F*HW][256], xn [B*F*HW][C] bf16 for the weight
// gradients; dbias_part [B][8][nblk][F][F] (cesm_relpos_bwd layout); dgamma (+)= sum dxn*xhat
// through dgamma_part [B*nblk][C].
int cesm_tblock_bwd(const void* x, const void* dy, const float* gamma, const float* mr, const float* lse,
                    const void* wqkv, const void* wqkv_t, const void* wout_t, const float* bias, const float* rot,
                    void* dx, void* dqkv, void* o, void* xn, float* dbias_part, float* dgamma, float* dgamma_part,
                    void* wimg, int nblk, int B, int F, int HW, int C, float scale, int accumulate,
                    hipStream_t stream) {
  if (F < 1 || F > 16 || nblk < 1) return CESM_EUNSUPPORTED;
  dim3 grid(nblk, B);
  if (C <= 256) {
    bf16* iq = (bf16*)wimg;
    bf16* iqt = iq + 768 * C;
    bf16* iot = iqt + 768 * C;
    frag_image(wqkv, iq, 768, C, stream);
    frag_image(wqkv_t, iqt, C, QKV, stream);
    frag_image(wout_t, iot, INNER, C, stream);
    wqkv = iq;
    wqkv_t = iqt;
    wout_t = iot;
  }
  switch (C) {
    case 64:
    case 128:
    case 256: {
      const int rc = C == 64 ? tw_bwd_launch<64>(x, dy, gamma, mr, lse, wqkv, wqkv_t, wout_t, bias, rot, dx, dqkv, o, xn,
                                                 dbias_part, dgamma_part, grid, F, HW, scale, stream)
                   : C == 128 ? tw_bwd_launch<128>(x, dy, gamma, mr, lse, wqkv, wqkv_t, wout_t, bias, rot, dx, dqkv, o, xn,
                                                   dbias_part, dgamma_part, grid, F, HW, scale, stream)
                              : tw_bwd_launch<256>(x, dy, gamma, mr, lse, wqkv, wqkv_t, wout_t, bias, rot, dx, dqkv, o, xn,
                                                   dbias_part, dgamma_part, grid, F, HW, scale, stream);
      if (rc) return rc;
      break;
    }
    case 512:
      tblock_bwd_kernel<512><<<grid, 256, 0, stream>>>(
          (const bf16*)x, (const bf16*)dy, gamma, mr, lse, (const bf16*)wqkv, (const bf16*)wqkv_t,
          (const bf16*)wout_t, bias, rot, (bf16*)dx, (bf16*)dqkv, (bf16*)o, (bf16*)xn, dbias_part, dgamma_part, F, HW,
          scale);
      break;
    default:
      return CESM_EUNSUPPORTED;
  }
  if (dgamma) tb_sum_rows_kernel<<<C, 64, 0, stream>>>(dgamma_part, dgamma, B * nblk, C, accumulate);
  return cesm_launch_status();
}

// blocks of cesm_tblock_bwd_dw (one per CU, grid-stride over pixel groups); 0 = shape not supported
int cesm_tblock_bwd_dw_nblk(int B, int F, int HW, int C) {
  if (C != 64 || F < 1 || 4 * F > 16 * TH_NVMAX || B < 1 || HW < 1) return 0;
  const int ngroups = B * (int)cdiv(HW, 4);
  return std::min(ngroups, cesm_num_cus());
}

// Forward with gamma folded into the QKV weights (the forward of cesm_tblock_bwd_dw, C = 64): as
// cesm_tblock_fwd, but wqkv_f32 is the fp32 master weight [768][C]; the LN output fed to the GEMMs is xhat.
int cesm_tblock_fwd_fold(const void* x, const float* gamma, const float* wqkv_f32, const void* wout,
                         const float* bias, const float* rot, void* y, float* mr, float* lse, void* o, void* wimg,
                         int B, int F, int HW, int C, float scale, float eps, hipStream_t stream) {
  if (C != 64 || F < 1 || F > 16) return CESM_EUNSUPPORTED;
  bf16* iq = (bf16*)wimg;
  bf16* io = iq + 768 * C;
  frag_image_f32_kernel<<<(unsigned)cdiv((int64_t)768 * C / 8, 256), 256, 0, stream>>>(wqkv_f32, gamma, iq, 768, C, 0,
                                                                                      INNER, scale);  // q rows x scale
  frag_image(wout, io, C, INNER, stream);
  const int nv = (TW<64>::PW * F + 15) / 16;
  switch (nv) {
    case 1: tw_fwd_launch_nv<64, 1, true>(x, gamma, iq, io, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream); break;
    case 2: tw_fwd_launch_nv<64, 2, true>(x, gamma, iq, io, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream); break;
    case 3: tw_fwd_launch_nv<64, 3, true>(x, gamma, iq, io, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream); break;
    case 4: tw_fwd_launch_nv<64, 4, true>(x, gamma, iq, io, bias, rot, y, mr, lse, o, B, F, HW, scale, eps, stream); break;
    default: return CESM_EUNSUPPORTED;
  }
  return cesm_launch_status();
}

// Head-parallel fused backward of the temporal-attention block with in-kernel weight gradients (C = 64,
// 4F <= 48; the forward must be cesm_tblock_fwd_fold's).  dx [B*F*HW][C]; o (nullable) [B*F*HW][256] the attention
// output recomputed from the backward's P (the to_out weight gradient's input); dwqkv (+)= dW_qkv [768][C] and
// dgamma (+)= the LN gamma gradient (each nullable); dbias_part [8][nblk][F][F] (cesm_relpos_bwd with
// B = 1).  Workspaces: slab nblk*768*C floats, tmp 768*C floats, wimg (2*768 + 256)*C bf16.
int cesm_tblock_bwd_dw(const void* x, const void* dy, const float* mr, const float* lse, const float* wqkv_f32,
                       const float* gamma, const void* wout_t, const float* bias, const float* rot, void* dx, void* o,
                       float* dwqkv, float* dgamma, float* dbias_part, float* slab, float* tmp, void* wimg,
                       int nblk, int B, int F, int HW, int C, float scale, int accumulate, hipStream_t stream) {
  if (nblk < 1 || nblk != cesm_tblock_bwd_dw_nblk(B, F, HW, C)) return CESM_EUNSUPPORTED;
  if (o && (int64_t)F * HW * INNER >= ((int64_t)1 << 31)) return CESM_EUNSUPPORTED;  // 32-bit O row offsets per sample
  bf16* iq = (bf16*)wimg;
  bf16* iqt = iq + 768 * C;
  bf16* iot = iqt + 768 * C;
  const unsigned gi = (unsigned)cdiv((int64_t)768 * C / 8, 256);
  // W diag(gamma) and its transpose, the q rows times the attention scale (the kernel's q epilogues skip it)
  frag_image_f32_kernel<<<gi, 256, 0, stream>>>(wqkv_f32, gamma, iq, 768, C, 0, INNER, scale);
  frag_image_f32_kernel<<<gi, 256, 0, stream>>>(wqkv_f32, gamma, iqt, C, 768, 1, INNER, scale);
  frag_image(wout_t, iot, INNER, C, stream);
  const int nv = (4 * F + 15) / 16;
  const size_t sm = twh_smem(F, nv);
#define TWH_LAUNCH(NVv)                                                                                           \
  allow_smem(twh_bwd_kernel<NVv>, sm);                                                                            \
  twh_bwd_kernel<NVv><<<nblk, 512, sm, stream>>>((const bf16*)x, (const bf16*)dy, mr, lse, iq, iqt, iot, bias, rot, \
                                                 (bf16*)dx, (bf16*)o, slab, dbias_part, B, F, HW, scale)
  switch (nv) {
    case 1: TWH_LAUNCH(1); break;
    case 2: TWH_LAUNCH(2); break;
    case 3: TWH_LAUNCH(3); break;
    default: return CESM_EUNSUPPORTED;
  }
#undef TWH_LAUNCH
  const int64_t nel = (int64_t)768 * C;
  twh_dw_reduce_kernel<<<twh_dw_reduce_grid(nel), 256, 0, stream>>>(slab, nblk, wqkv_f32, gamma, dwqkv, tmp, 768, C,
                                                                    accumulate, INNER, scale);
  if (dgamma) twh_dgamma_kernel<<<C, 256, 0, stream>>>(tmp, dgamma, 768, C, accumulate);
  return cesm_launch_status();
}

}  // extern "C"
