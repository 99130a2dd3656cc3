// Fused spatial linear attention block (bf16, C = 64): Residual(PreNorm(SpatialLinearAttention))
// (video_net.py:313-347, :69-98).  Per frame n, head h (8 x 32):
//   xn = LN(x);  q,k,v = W_{q,k,v} xn
//   q~[d,p] = scale * softmax_d(q)[d,p]      k~[d,p] = softmax_p(k)[d,p] = exp(k - M_d) / Z_d
//   ctx[d,e] = sum_p k~[d,p] v[e,p]          o[e,p] = sum_d ctx[d,e] q~[d,p]
//   y = x + W_o o + b_o
// Forward = three launches, none of which writes a per-pixel intermediate:
//   slaf_stats   (8 waves = 8 heads, xn tile in LDS): online-softmax partials per block:
//                m_d, s_d = sum exp(k - m), u^T[e][d] = sum_p v[e,p] exp(k[d,p] - m_d)
//   slaf_combine per (frame, head): M, Z, ctx; ctx also written as ready-to-load MFMA A fragments
//   slaf_out     (wave = 64 pixels, all heads): LN -> q -> softmax_d -> o = ctx^T q~ -> y, with q~ and o
//                kept in registers: the MFMA D layout (lane (g, i): rows 4g..4g+3 of a 16-row tile,
//                column i) is fed back as a B operand through the k-slot map
//                slot (g, j<4) <-> k = 4g + j,  slot (g, 4+j) <-> k = 16 + 4g + j.
#include "common.h"
#include "cesm_hip.h"

namespace {

constexpr int NH = 8, DH = 32, INNER = 256, QKV = 768;
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}
__device__ __forceinline__ bf16x8 ld16(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
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
// k index of slot (g, j) of the k-slot map
__device__ __forceinline__ int kslot(int g, int j) { return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4); }
// B/A operand from two D-layout 16-row tiles (rows 0..15 -> slots 0..3, rows 16..31 -> slots 4..7)
__device__ __forceinline__ bf16x8 pack_kslot(const float* t0, const float* t1) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (bf16)t0[j];
    r[4 + j] = (bf16)t1[j];
  }
  return r;
}

// ---------------------------------------------------------------------------------------------------
// slaf_stats: grid (nblk, Nf), 512 threads (wave h = head h).  Block b of frame n handles 64-pixel
// sub-chunks [b*spb, (b+1)*spb).  Partial layout per (n, b, h): m[32] | s[32] | uT[32 e][32 d].
// ---------------------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(512) void slaf_stats_kernel(const bf16* __restrict__ x, const float* __restrict__ gamma,
                                                         const bf16* __restrict__ wqkv, float* __restrict__ part,
                                                         int HW, int spb, float eps) {
  constexpr int KS = C / 32, XLD = C + 8, L = C / 8, PPP = 512 / L;  // LN lanes per pixel, pixels per pass
  __shared__ __attribute__((aligned(16))) bf16 xs[64 * XLD];
  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int n = blockIdx.y;
  const int nsc = (HW + 63) / 64;
  const int sc0 = blockIdx.x * spb, sc1 = min(nsc, sc0 + spb);
  const bf16* xf = x + (int64_t)n * HW * C;

  // B fragments W[ch][ci] of this head's k and v rows
  bf16x8 wk[2][KS], wv[2][KS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      wk[t][ks] = ld16(wqkv + (int64_t)(INNER + h * DH + t * 16 + lr) * C + ks * 32 + lg * 8);
      wv[t][ks] = ld16(wqkv + (int64_t)(2 * INNER + h * DH + t * 16 + lr) * C + ks * 32 + lg * 8);
    }
  float m[2] = {-INFINITY, -INFINITY}, s[2] = {0.f, 0.f};  // d = t*16 + lr
  f32x4 uT[2][2];                                           // [e tile][d tile]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) uT[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  // the next 64-pixel chunk's x vectors are loaded into registers while the current one is consumed
  constexpr int NPASS = 64 / PPP;
  const int sub = tid % L;
  bf16x8 xr[NPASS];
  auto gload = [&](int sc) {
#pragma unroll
    for (int k = 0; k < NPASS; ++k) {
      const int p = sc * 64 + k * PPP + tid / L;
      xr[k] = *reinterpret_cast<const bf16x8*>(xf + (int64_t)(p < HW ? p : 0) * C + sub * 8);  // row 0 past HW
    }
  };
  if (sc0 < sc1) gload(sc0);
  float gm8[8];
  load8(gamma + sub * 8, gm8);

  for (int sc = sc0; sc < sc1; ++sc) {
    const int p0 = sc * 64;
    __syncthreads();
    // LN of 64 pixels into xs (rows beyond HW zero)
    {
#pragma unroll
      for (int pp0 = 0; pp0 < 64; pp0 += PPP) {
        const int pl = pp0 + tid / L;
        const int p = p0 + pl;
        float a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = p < HW ? (float)xr[pp0 / PPP][i] : 0.f;
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) sm += a[i];
        sm = group_sum(sm, L);
        const float mean = sm / C;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float d = a[i] - mean; q = fmaf(d, d, q); }
        q = group_sum(q, L);
        const float rstd = 1.f / sqrtf(q / C + eps);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = p < HW ? (a[i] - mean) * rstd * gm8[i] : 0.f;
        store8(xs + pl * XLD + sub * 8, a);
      }
    }
    __syncthreads();
    if (sc + 1 < sc1) gload(sc + 1);
    // k, v of this head for 64 pixels: D[px = vt*16 + 4g + r][ch = t*16 + i]
    f32x4 kk[4][2], vv[4][2];
#pragma unroll
    for (int vt = 0; vt < 4; ++vt) {
      bf16x8 af[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) af[ks] = ld16(xs + (vt * 16 + lr) * XLD + ks * 32 + lg * 8);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 ak = z4, av = z4;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          ak = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], wk[t][ks], ak, 0, 0, 0);
          av = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], wv[t][ks], av, 0, 0, 0);
        }
        kk[vt][t] = ak;
        vv[vt][t] = av;
      }
    }
    // online softmax over pixels, per d = t*16 + lr
    float corr[2], mn[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float lm = -INFINITY;
#pragma unroll
      for (int vt = 0; vt < 4; ++vt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (p0 + vt * 16 + lg * 4 + r < HW) lm = fmaxf(lm, kk[vt][t][r]);
      lm = grp4_max(lm);
      mn[t] = fmaxf(m[t], lm);
      corr[t] = m[t] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m[t] - mn[t]) * LOG2E);
    }
    float pe[4][2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float ps = 0.f;
#pragma unroll
      for (int vt = 0; vt < 4; ++vt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = p0 + vt * 16 + lg * 4 + r < HW;
          pe[vt][t][r] = ok ? __builtin_amdgcn_exp2f((kk[vt][t][r] - mn[t]) * LOG2E) : 0.f;
          ps += pe[vt][t][r];
        }
      ps = grp4_sum(ps);
      s[t] = s[t] * corr[t] + ps;
      m[t] = mn[t];
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int r = 0; r < 4; ++r) uT[e][t][r] *= corr[t];
    }
    // uT[e][d] += sum_p v[p][e] p[p][d]   (two 32-pixel k-steps from tile pairs (0,1), (2,3))
#pragma unroll
    for (int kp = 0; kp < 2; ++kp) {
      const int va = 2 * kp, vb = 2 * kp + 1;
      bf16x8 Av[2], Bp[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        float a0[4] = {vv[va][t][0], vv[va][t][1], vv[va][t][2], vv[va][t][3]};
        float a1[4] = {vv[vb][t][0], vv[vb][t][1], vv[vb][t][2], vv[vb][t][3]};
        Av[t] = pack_kslot(a0, a1);
        Bp[t] = pack_kslot(pe[va][t], pe[vb][t]);
      }
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int t = 0; t < 2; ++t) uT[e][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Av[e], Bp[t], uT[e][t], 0, 0, 0);
    }
  }
  float* o = part + (((int64_t)n * gridDim.x + blockIdx.x) * NH + h) * (64 + 1024);
  if (lg == 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      o[t * 16 + lr] = m[t];
      o[32 + t * 16 + lr] = s[t];
    }
  }
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[64 + (e * 16 + lg * 4 + r) * 32 + t * 16 + lr] = uT[e][t][r];
}

// ---------------------------------------------------------------------------------------------------
// slaf_combine: grid (Nf * 8), 256 threads.  mz[n][h][d] = (M, Z); ctx32[n][h][d][e];
// A-fragment images (bf16, [n][h][tile][lane][8]):  actT rows e / k = d  (o = ctx^T q~),
//                                                     actx rows d / k = e  (dq~ = ctx do).
// ---------------------------------------------------------------------------------------------------
constexpr int SLAF_NBLK_MAX = 128;  // partial blocks per frame (cesm_slaf_nblk caps it)

__global__ __launch_bounds__(256) void slaf_combine_kernel(const float* __restrict__ part, int nblk,
                                                           float* __restrict__ mz, float* __restrict__ ctx32,
                                                           bf16* __restrict__ actT, bf16* __restrict__ actx) {
  __shared__ float sM[32], sZ[32];
  __shared__ float red[8][33];
  __shared__ __attribute__((aligned(16))) float sw[SLAF_NBLK_MAX][32];  // exp(m_b[d] - M[d])
  __shared__ float sc[32][33];  // [d][e]
  const int nh = blockIdx.x, n = nh / NH, h = nh % NH;
  const int tid = threadIdx.x;
  const float* pb = part + ((int64_t)n * nblk * NH + h) * (64 + 1024);
  const int64_t bstride = (int64_t)NH * (64 + 1024);
  // M_d = max_b m_b[d], Z_d = sum_b exp(m_b[d] - M_d) s_b[d]: thread (d, slice of 8 over b)
  const int d = tid & 31, sl = tid >> 5;
  float M = -INFINITY;
  for (int b = sl; b < nblk; b += 8) M = fmaxf(M, pb[b * bstride + d]);
  red[sl][d] = M;
  __syncthreads();
  if (tid < 32) {
    float m = red[0][tid];
#pragma unroll
    for (int k = 1; k < 8; ++k) m = fmaxf(m, red[k][tid]);
    sM[tid] = m;
  }
  __syncthreads();
  M = sM[d];
  float Z = 0.f;
  for (int b = sl; b < nblk; b += 8) {
    const float mb = pb[b * bstride + d];
    const float w = mb == -INFINITY ? 0.f : expf(mb - M);
    sw[b][d] = w;
    Z = fmaf(w, pb[b * bstride + 32 + d], Z);
  }
  __syncthreads();
  red[sl][d] = Z;
  __syncthreads();
  if (tid < 32) {
    float z = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) z += red[k][tid];
    sZ[tid] = z;
    mz[((int64_t)nh * 32 + tid) * 2] = sM[tid];
    mz[((int64_t)nh * 32 + tid) * 2 + 1] = z;
  }
  __syncthreads();
  // U[e][d] = sum_b w_b[d] u_b[e][d]: thread owns idx = 4 tid .. 4 tid + 3 (e = idx / 32, d = idx % 32)
  const int e = (tid * 4) >> 5, d0 = (tid * 4) & 31;
  f32x4 U = {0.f, 0.f, 0.f, 0.f};
  int b = 0;
  for (; b + 4 <= nblk; b += 4) {
    f32x4 u[4], w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      u[k] = *reinterpret_cast<const f32x4*>(pb + (b + k) * bstride + 64 + tid * 4);
      w[k] = *reinterpret_cast<const f32x4*>(&sw[b + k][d0]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) U += w[k] * u[k];
  }
  for (; b < nblk; ++b) U += *reinterpret_cast<const f32x4*>(&sw[b][d0]) * *reinterpret_cast<const f32x4*>(pb + b * bstride + 64 + tid * 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float zd = sZ[d0 + i];
    // Z >= 1 for every frame (the maximum's own term is exp(0)); no guard: a `Z > 0 ?` select turned a NaN Z into a
    // zero context (a NaN at one pixel vanished from the frame instead of reaching every pixel, as in the reference)
    const float c = U[i] / zd;
    sc[d0 + i][e] = c;
    ctx32[((int64_t)nh * 32 + d0 + i) * 32 + e] = c;
  }
  __syncthreads();
  // fragment images: 2 tiles x 64 lanes x 8
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + i * 256;  // (tile, lane, j) over 2*64*4 pairs of slots
    const int tile = idx >> 8, lane = (idx >> 2) & 63, jp = idx & 3;
    const int g = lane >> 4, l16 = lane & 15;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = jp * 2 + jj;
      const int k = kslot(g, j);
      const int row = tile * 16 + l16;
      const int64_t o = (((int64_t)nh * 2 + tile) * 64 + lane) * 8 + j;
      actT[o] = (bf16)sc[k][row];  // rows e, k = d
      actx[o] = (bf16)sc[row][k];  // rows d, k = e
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// slaf_out: wave = 16*NV pixels of one frame, all heads; grid (cdiv(HW, 64*NV), Nf), 256 threads.
// ---------------------------------------------------------------------------------------------------
typedef unsigned int sl_u32x2 __attribute__((ext_vector_type(2)));
template <int C, int NV>
// slaf_out capped at 256 registers (waves_per_eu 2: VGPR-form MFMAs, no AGPR stash)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void slaf_out_kernel(const bf16* __restrict__ x, const float* __restrict__ gamma,
                                                       const bf16* __restrict__ wqkv, const bf16* __restrict__ wout,
                                                       const float* __restrict__ bout, const bf16* __restrict__ actT,
                                                       bf16* __restrict__ y, bf16* __restrict__ o_out, int HW, float scale, float eps) {
  constexpr int KS = C / 32, CT = C / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int n = blockIdx.y;
  const int p0 = (blockIdx.x * 4 + wid) * 16 * NV;
  if (p0 >= HW) return;
  const bf16* xb = x + (int64_t)n * HW * C;
  // LN on the B fragments: lane (g, i) holds pixel p0 + vt*16 + i, channels ks*32 + 8g..8g+7
  float gm[KS][8];  // gamma hoisted: under the lane predicate each element was its own load + vmcnt(0)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) load8(gamma + ks * 32 + lg * 8, gm[ks]);
  bf16x8 xf[NV][KS];
#pragma unroll
  for (int vt = 0; vt < NV; ++vt) {
    const int p = p0 + vt * 16 + lr;
    const bool ok = p < HW;
    float a[KS][8];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {  // unpredicated loads (row 0 past HW), then selected
      load8(xb + (int64_t)(ok ? p : 0) * C + ks * 32 + lg * 8, a[ks]);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[ks][i] = ok ? a[ks][i] : 0.f;
    }
    float sm = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i) sm += a[ks][i];
    const float mean = grp4_sum(sm) / C;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float d = a[ks][i] - mean; q = fmaf(d, d, q); }
    const float rstd = 1.f / sqrtf(grp4_sum(q) / C + eps);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i) xf[vt][ks][i] = (bf16)(ok ? (a[ks][i] - mean) * rstd * gm[ks][i] : 0.f);
  }
  f32x4 yacc[CT][NV];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) yacc[ct][vt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  const bf16* actn = actT + (int64_t)n * NH * 2 * 64 * 8;

  for (int h = 0; h < NH; ++h) {
    bf16x8 wq[2][KS];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) wq[t][ks] = ld16(wqkv + (int64_t)(h * DH + t * 16 + lr) * C + ks * 32 + lg * 8);
    bf16x8 at[2];
#pragma unroll
    for (int et = 0; et < 2; ++et) at[et] = ld16(actn + ((h * 2 + et) * 64 + lane) * 8);
    // W_o[co][h*32 + kslot(g, j)] fragments
    bf16x8 wo[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const bf16* src = wout + (int64_t)(ct * 16 + lr) * INNER + h * DH + lg * 4;
      const s16x4 lo = *reinterpret_cast<const s16x4*>(src);
      const s16x4 hi = *reinterpret_cast<const s16x4*>(src + 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wo[ct][j] = __builtin_bit_cast(bf16, (short)lo[j]);
        wo[ct][4 + j] = __builtin_bit_cast(bf16, (short)hi[j]);
      }
    }
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      float qv[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 a = z4;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wq[t][ks], xf[vt][ks], a, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) qv[t][r] = a[r];
      }
      // softmax over d (rows t*16 + 4g + r) for pixel lr
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, qv[t][r]);
      mx = grp4_max(mx);
      float sm = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          qv[t][r] = __builtin_amdgcn_exp2f((qv[t][r] - mx) * LOG2E);
          sm += qv[t][r];
        }
      const float inv = scale * __builtin_amdgcn_rcpf(grp4_sum(sm));
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) qv[t][r] *= inv;
      const bf16x8 qb = pack_kslot(qv[0], qv[1]);
      // o^T = ctx^T q~  -> rows e
      float ov[2][4];
#pragma unroll
      for (int et = 0; et < 2; ++et) {
        const f32x4 o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[et], qb, z4, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) ov[et][r] = o[r];
      }
      const bf16x8 ob = pack_kslot(ov[0], ov[1]);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) yacc[ct][vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wo[ct], ob, yacc[ct][vt], 0, 0, 0);
      if (o_out) {  // O for the to_out weight gradient (the backward then skips its emission)
        const int p = p0 + vt * 16 + lr;
        if (p < HW) {
#pragma unroll
          for (int et = 0; et < 2; ++et) stnt4(o_out + ((int64_t)n * HW + p) * INNER + h * DH + et * 16 + lg * 4, ov[et]);
        }
      }
    }
  }
  // y = x + W_o o + b_o
  // every residual / bias load before the first y store, the stores branch-free through a buffer resource over frame
  // n (pixels past HW go to an out-of-range offset, which the hardware drops): vmcnt retires in issue order, so a load
  // behind a store waits for it (round 5: SLA forward 2.50 -> 2.48 ms, profiles/r5f_epilogue_loads_first_tb.txt)
  {
    const __amdgpu_buffer_rsrc_t yrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(y + (int64_t)n * HW * C), (short)0, HW * C * 2, 0x00020000);
    f32x4 bo[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) bo[ct] = *reinterpret_cast<const f32x4*>(bout + ct * 16 + lg * 4);
    bf16x4 xr[NV][CT];
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      const int p = p0 + vt * 16 + lr;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        xr[vt][ct] = *reinterpret_cast<const bf16x4*>(xb + (int64_t)(p < HW ? p : 0) * C + ct * 16 + lg * 4);
    }
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      const int p = p0 + vt * 16 + lr;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)((float)xr[vt][ct][r] + yacc[ct][vt][r] + bo[ct][r]);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(sl_u32x2, o), yrs,
                                              p < HW ? (p * C + ct * 16 + lg * 4) * 2 : 0x7ffffff0, 0, 0);
      }
    }
  }
}

// ===================================================================================================
// Backward.  With do = W_o^T dy:
//   dq~ = ctx do,  dctx = sum_p q~ do^T,  dq = scale sm (dq~ - sum_d sm dq~)       (sm = softmax_d q)
//   dk~ = dctx v,  dv = dctx^T k~,       dk = k~ (dk~ - G),  G_d = sum_p k~ dk~ = sum_e dctx[d,e] ctx[d,e]
//   dxn = W_q^T dq + W_k^T dk + W_v^T dv -> LN backward (+ dy residual)
// slab_dctx (8 waves = heads, non-transposed tiles) -> slab_combine -> slab_dx (per wave, all heads).
// ===================================================================================================

// max / sum over the 16 lanes of a row with DPP (quad_perm xor1, xor2, row_half_mirror, row_mirror)
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

// grid (nblk, Nf), 512 threads; partial per (n, b, h): dctx[32 d][32 e]
// DWO (C = 64, the in-kernel-dW backward): also the to_out weight / bias gradient inputs without the forward's
// 256-channel O: O_h = ctx_h^T q~_h per pixel, so dW_out[:, h] = (sum_px dy q~_h^T) ctx_h — the per-block
// M_h = sum_px dy q~_h^T (64 x 32, K = pixels on MFMA: dy^T by k-slot transposed reads from the staged tile, q~ the
// packed fragment the dctx product already uses) goes to partm [n][blk][h][64][32], sum_px dy to partb [n][blk][C]
template <int C, bool DWO = false>
__global__ __launch_bounds__(512) void slab_dctx_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                        const float* __restrict__ gamma, const bf16* __restrict__ wqkv,
                                                        const bf16* __restrict__ wout_t, float* __restrict__ part,
                                                        int HW, int spb, float scale, float eps,
                                                        float* __restrict__ partm = nullptr,
                                                        float* __restrict__ partb = nullptr) {
  constexpr int KS = C / 32, XLD = C + 8, L = C / 8, PPP = 512 / L;
  static_assert(!DWO || C == 64, "to_out gradient inputs at C = 64 only");
  __shared__ __attribute__((aligned(16))) bf16 xs[64 * XLD];
  __shared__ __attribute__((aligned(16))) bf16 ds[64 * XLD];
  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int n = blockIdx.y;
  const int nsc = (HW + 63) / 64;
  const int sc0 = blockIdx.x * spb, sc1 = min(nsc, sc0 + spb);
  const bf16* xb = x + (int64_t)n * HW * C;
  const bf16* db = dy + (int64_t)n * HW * C;
  bf16x8 wq[2][KS], wo[2][KS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      wq[t][ks] = ld16(wqkv + (int64_t)(h * DH + t * 16 + lr) * C + ks * 32 + lg * 8);
      wo[t][ks] = ld16(wout_t + (int64_t)(h * DH + t * 16 + lr) * C + ks * 32 + lg * 8);
    }
  f32x4 dc[2][2];  // [d tile][e tile]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) dc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 macc[4][2];  // DWO: M_h [c tile][d tile]
  float bsum[8];     // DWO: this thread's sum of dy over its pixels, channels sub*8 ..
#pragma unroll
  for (int a = 0; a < 4; ++a) macc[a][0] = macc[a][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i) bsum[i] = 0.f;
  // the next 64-pixel chunk's x / dy vectors are loaded into registers while the current one is consumed
  constexpr int NPASS = 64 / PPP;
  const int sub = tid % L;
  bf16x8 xr[NPASS], dr[NPASS];
  auto gload = [&](int sc) {
#pragma unroll
    for (int k = 0; k < NPASS; ++k) {
      const int p = sc * 64 + k * PPP + tid / L;
      const int64_t ps = p < HW ? p : 0;  // unpredicated loads (row 0 past HW), selected when staged
      xr[k] = *reinterpret_cast<const bf16x8*>(xb + ps * C + sub * 8);
      dr[k] = *reinterpret_cast<const bf16x8*>(db + ps * C + sub * 8);
    }
  };
  if (sc0 < sc1) gload(sc0);
  float gm8[8];
  load8(gamma + sub * 8, gm8);
  for (int sc = sc0; sc < sc1; ++sc) {
    const int p0 = sc * 64;
    __syncthreads();
    {
#pragma unroll
      for (int pp0 = 0; pp0 < 64; pp0 += PPP) {
        const int pl = pp0 + tid / L;
        const int p = p0 + pl;
        float a[8], d8[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) { a[i] = (float)xr[pp0 / PPP][i]; d8[i] = (float)dr[pp0 / PPP][i]; }
#pragma unroll
        for (int i = 0; i < 8; ++i) { a[i] = p < HW ? a[i] : 0.f; d8[i] = p < HW ? d8[i] : 0.f; }
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) sm += a[i];
        sm = group_sum(sm, L);
        const float mean = sm / C;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float d = a[i] - mean; q = fmaf(d, d, q); }
        q = group_sum(q, L);
        const float rstd = 1.f / sqrtf(q / C + eps);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = p < HW ? (a[i] - mean) * rstd * gm8[i] : 0.f;
        if constexpr (DWO) {
#pragma unroll
          for (int i = 0; i < 8; ++i) bsum[i] += d8[i];
        }
        store8(xs + pl * XLD + sub * 8, a);
        store8(ds + pl * XLD + sub * 8, d8);
      }
    }
    __syncthreads();
    if (sc + 1 < sc1) gload(sc + 1);
    float qt[4][2][4], dv[4][2][4];  // q~ [px tile][d tile][r], do [px tile][e tile][r]
#pragma unroll
    for (int vt = 0; vt < 4; ++vt) {
      bf16x8 ax[KS], ad[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        ax[ks] = ld16(xs + (vt * 16 + lr) * XLD + ks * 32 + lg * 8);
        ad[ks] = ld16(ds + (vt * 16 + lr) * XLD + ks * 32 + lg * 8);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 aq = z4, ao = z4;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          aq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[ks], wq[t][ks], aq, 0, 0, 0);
          ao = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad[ks], wo[t][ks], ao, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) { qt[vt][t][r] = aq[r]; dv[vt][t][r] = ao[r]; }
      }
      // softmax over d (lanes of the row x 2 tiles) for pixel vt*16 + 4g + r
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float mx = row16_max(fmaxf(qt[vt][0][r], qt[vt][1][r]));
        const float e0 = __builtin_amdgcn_exp2f((qt[vt][0][r] - mx) * LOG2E);
        const float e1 = __builtin_amdgcn_exp2f((qt[vt][1][r] - mx) * LOG2E);
        const float inv = scale * __builtin_amdgcn_rcpf(row16_sum(e0 + e1));
        qt[vt][0][r] = e0 * inv;
        qt[vt][1][r] = e1 * inv;
      }
    }
#pragma unroll
    for (int kp = 0; kp < 2; ++kp) {
      const int va = 2 * kp, vb = 2 * kp + 1;
      bf16x8 Aq[2], Bd[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        Aq[t] = pack_kslot(qt[va][t], qt[vb][t]);
        Bd[t] = pack_kslot(dv[va][t], dv[vb][t]);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) dc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Aq[a], Bd[b], dc[a][b], 0, 0, 0);
      if constexpr (DWO) {
        // dy^T as the A operand: lane (i = channel, g) element e = dy[px of k-slot (g, e)][ct*16 + i]
        const int g = lane >> 4, qq = (lane >> 2) & 3, pq = lane & 3;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (LDS_PTR(s16x4))(ds + (va * 16 + 4 * g + qq) * XLD + ct * 16 + 4 * pq));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (LDS_PTR(s16x4))(ds + (vb * 16 + 4 * g + qq) * XLD + ct * 16 + 4 * pq));
          bf16x8 ady;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ady[e] = __builtin_bit_cast(bf16, (short)lo[e]);
            ady[4 + e] = __builtin_bit_cast(bf16, (short)hi[e]);
          }
#pragma unroll
          for (int t = 0; t < 2; ++t) macc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ady, Aq[t], macc[ct][t], 0, 0, 0);
        }
      }
    }
  }
  if constexpr (DWO) {
    float* om = partm + (((int64_t)n * gridDim.x + blockIdx.x) * NH + h) * 2048;  // [c][d]
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) om[(ct * 16 + lg * 4 + r) * 32 + t * 16 + lr] = macc[ct][t][r];
    // bias: threads sharing sub (lanes l, l^8, l^16, ... and the 8 waves) summed in a fixed order
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) bsum[i] += __shfl_xor(bsum[i], o, 64);
    __syncthreads();
    float* sb = reinterpret_cast<float*>(xs);  // [8 waves][64 channels]
    if (lane < 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) sb[h * 64 + lane * 8 + i] = bsum[i];
    }
    __syncthreads();
    if (tid < 64) {
      float b = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) b += sb[w * 64 + tid];
      partb[((int64_t)n * gridDim.x + blockIdx.x) * 64 + tid] = b;
    }
  }
  float* o = part + (((int64_t)n * gridDim.x + blockIdx.x) * NH + h) * 1024;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(a * 16 + lg * 4 + r) * 32 + b * 16 + lr] = dc[a][b][r];
}

// to_out weight gradient from slab_dctx<64, true>'s partials: per (frame n, head h) R[c][e] = sum_d
// (sum_blk M[n][blk][h][c][d]) ctx32[n][h][d][e]  (grid Nf * 8, 256 threads; fixed-order sums)
__global__ __launch_bounds__(256) void slab_dwout_frame_kernel(const float* __restrict__ partm, int nblk,
                                                               const float* __restrict__ ctx32, float* __restrict__ R) {
  __shared__ float sm[64][33];
  __shared__ float sc[32][33];
  const int nh = blockIdx.x, n = nh / NH, h = nh % NH, tid = threadIdx.x;
  for (int i = tid; i < 1024; i += 256) sc[i >> 5][i & 31] = ctx32[(int64_t)nh * 1024 + i];
  const float* pm = partm + ((int64_t)n * nblk * NH + h) * 2048;
  for (int i = tid; i < 2048; i += 256) {
    float m = 0.f;
#pragma unroll 4
    for (int b = 0; b < nblk; ++b) m += pm[(int64_t)b * NH * 2048 + i];
    sm[i >> 5][i & 31] = m;
  }
  __syncthreads();
  for (int i = tid; i < 2048; i += 256) {
    const int c = i >> 5, e = i & 31;
    float r = 0.f;
#pragma unroll 8
    for (int d = 0; d < 32; ++d) r = fmaf(sm[c][d], sc[d][e], r);
    R[(int64_t)nh * 2048 + i] = r;
  }
}

// dwout [C = 64][256] (+)= sum over frames of R[n][h][c][e] at column h*32 + e (thread per output element)
__global__ __launch_bounds__(256) void slab_dwout_sum_kernel(const float* __restrict__ R, int Nf, float* __restrict__ dwout,
                                                             int accumulate) {
  const int idx = blockIdx.x * 256 + threadIdx.x;  // (c, h, e)
  if (idx >= 64 * 256) return;
  const int c = idx >> 8, k = idx & 255, h = k >> 5, e = k & 31;
  float s = 0.f;
#pragma unroll 8
  for (int n = 0; n < Nf; ++n) s += R[((int64_t)(n * NH + h) * 64 + c) * 32 + e];
  dwout[idx] = accumulate ? dwout[idx] + s : s;
}

// grid (Nf * 8), 256 threads: dctx = sum of partials; G; A-fragment images adc (rows d / k = e) and
// adcT (rows e / k = d)
__global__ __launch_bounds__(256) void slab_combine_kernel(const float* __restrict__ part, int nblk,
                                                           const float* __restrict__ ctx32, const float* __restrict__ mz,
                                                           float* __restrict__ kimg, bf16* __restrict__ adc,
                                                           bf16* __restrict__ adcT) {
  __shared__ float sd[32][33];
  __shared__ float sg[32][9];
  __shared__ float sG[32];
  const int nh = blockIdx.x, n = nh / NH, h = nh % NH;
  const int tid = threadIdx.x;
  const float* pb = part + ((int64_t)n * nblk * NH + h) * 1024;
  const int64_t bstride = (int64_t)NH * 1024;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid * 4 + i, d = idx >> 5, e = idx & 31;
    float a = 0.f;
    for (int b = 0; b < nblk; ++b) a += pb[b * bstride + idx];
    sd[d][e] = a;
  }
  __syncthreads();
  {  // G_d = sum_e dctx[d][e] ctx[d][e]: thread (d, 8 groups of 4 e)
    const int d = tid >> 3, eg = tid & 7;
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) a += sd[d][eg * 4 + j] * ctx32[((int64_t)nh * 32 + d) * 32 + eg * 4 + j];
    sg[d][eg] = a;
  }
  __syncthreads();
  if (tid < 32) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) a += sg[tid][j];
    sG[tid] = a;
  }
  __syncthreads();
  // per-lane image for slab_dx: lane (g, i), d = t*16 + 4g + r:
  //   [t*4 + r] = M_d log2(e) + log2(Z_d)  (k~ = exp2(k log2(e) - it)),  [8 + t*4 + r] = G_d
  if (tid < 64) {
    const int g = tid >> 4;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = t * 16 + 4 * g + r;
        const float M = mz[((int64_t)nh * 32 + d) * 2], Z = mz[((int64_t)nh * 32 + d) * 2 + 1];
        kimg[((int64_t)nh * 64 + tid) * 16 + t * 4 + r] = M * LOG2E + log2f(Z);
        kimg[((int64_t)nh * 64 + tid) * 16 + 8 + t * 4 + r] = sG[d];
      }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + i * 256;
    const int tile = idx >> 8, lane = (idx >> 2) & 63, jp = idx & 3;
    const int g = lane >> 4, l16 = lane & 15;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = jp * 2 + jj;
      const int k = kslot(g, j);
      const int row = tile * 16 + l16;
      const int64_t o = (((int64_t)nh * 2 + tile) * 64 + lane) * 8 + j;
      adc[o] = (bf16)sd[row][k];   // rows d, k = e
      adcT[o] = (bf16)sd[k][row];  // rows e, k = d
    }
  }
}

// slab_dx: wave = 16*NV pixels of one frame, all heads.  grid (cdiv(HW, 64*NV), Nf), 256 threads,
// dynamic LDS: 2C floats (dgamma accumulator, LN gamma) + 4 waves x [16*NV][DQLD] bf16 (this head's dq|dk|dv).
constexpr int DQLD = 104;
template <int C, int NV>
__global__ __launch_bounds__(256, 2) void slab_dx_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, const float* __restrict__ gamma,
    const bf16* __restrict__ wqkv, const bf16* __restrict__ wqkv_t, const bf16* __restrict__ wout_t,
    const float* __restrict__ kimg, const bf16* __restrict__ actT,
    const bf16* __restrict__ actx, const bf16* __restrict__ adc, const bf16* __restrict__ adcT,
    bf16* __restrict__ dx, bf16* __restrict__ dqkv_out, bf16* __restrict__ o_out, bf16* __restrict__ xn_out,
    float* __restrict__ dgamma_part, int HW, float scale, float eps) {
  constexpr int KS = C / 32, CT = C / 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // per-wave dgamma accumulators [4][C] (each written by one wave, lanes on distinct channels, summed in a
  // fixed order at the end: the block's partial is the same on every run — LDS float atomics across waves
  // were not)
  float* sgm = smem;  // [C] LN gamma (LDS reads do not queue behind the emission stores)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  float* sg = smem + C + wid * C;
  bf16* sq = reinterpret_cast<bf16*>(smem + 5 * C) + wid * 16 * NV * DQLD;
  for (int e = tid; e < 4 * C; e += 256) smem[C + e] = 0.f;
  for (int e = tid; e < C; e += 256) sgm[e] = gamma[e];
  __syncthreads();
  const int n = blockIdx.y;
  const int p0 = (blockIdx.x * 4 + wid) * 16 * NV;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  if (p0 < HW) {
    const int64_t rb = (int64_t)n * HW;
    bf16x8 xf[NV][KS];
    float mean[NV], rstd[NV];
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      const int p = p0 + vt * 16 + lr;
      const bool ok = p < HW;
      float a[KS][8];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {  // unpredicated loads (row 0 past HW), then selected
        load8(x + (rb + (ok ? p : 0)) * C + ks * 32 + lg * 8, a[ks]);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[ks][i] = ok ? a[ks][i] : 0.f;
      }
      float sm = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < 8; ++i) sm += a[ks][i];
      mean[vt] = grp4_sum(sm) / C;
      float q = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float d = a[ks][i] - mean[vt]; q = fmaf(d, d, q); }
      rstd[vt] = 1.f / sqrtf(grp4_sum(q) / C + eps);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          xf[vt][ks][i] = (bf16)(ok ? (a[ks][i] - mean[vt]) * rstd[vt] * sgm[ks * 32 + lg * 8 + i] : 0.f);
        if (ok && xn_out) *reinterpret_cast<bf16x8*>(xn_out + (rb + p) * C + ks * 32 + lg * 8) = xf[vt][ks];
      }
    }
    f32x4 dxacc[CT][NV];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) dxacc[ct][vt] = z4;
    // dy fragments, loaded once (not once per head)
    bf16x8 dyr[NV][KS];
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      const int p = p0 + vt * 16 + lr;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {  // unpredicated (row 0 past HW), then selected
        const bf16x8 v = ld16(dy + (rb + (p < HW ? p : 0)) * C + ks * 32 + lg * 8);
        dyr[vt][ks] = p < HW ? v : zero8();
      }
    }

    for (int h = 0; h < NH; ++h) {
      const int64_t fo = ((int64_t)(n * NH + h) * 2) * 64 * 8;
      bf16x8 aT[2], ax[2], ad[2], adT[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        aT[t] = ld16(actT + fo + (t * 64 + lane) * 8);
        ax[t] = ld16(actx + fo + (t * 64 + lane) * 8);
        ad[t] = ld16(adc + fo + (t * 64 + lane) * 8);
        adT[t] = ld16(adcT + fo + (t * 64 + lane) * 8);
      }
      // per-lane k-softmax offsets and G for d = t*16 + 4g + r (16-B loads of the combine's lane image)
      float Kofs[2][4], Gd[2][4];
      {
        const f32x4* ki = reinterpret_cast<const f32x4*>(kimg + ((int64_t)(n * NH + h) * 64 + lane) * 16);
        const f32x4 k0 = ki[0], k1 = ki[1], g0 = ki[2], g1 = ki[3];
#pragma unroll
        for (int r = 0; r < 4; ++r) { Kofs[0][r] = k0[r]; Kofs[1][r] = k1[r]; Gd[0][r] = g0[r]; Gd[1][r] = g1[r]; }
      }
      bf16x8 wh[4][2][KS];  // this head's q, k, v rows of W_qkv and do rows of W_out^T (fragment images)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
          for (int kind = 0; kind < 3; ++kind) wh[kind][t][ks] = ld_img(wqkv, kind * 16 + h * 2 + t, KS, ks, lane);
          wh[3][t][ks] = ld_img(wout_t, h * 2 + t, KS, ks, lane);
        }
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) {
        const int p = p0 + vt * 16 + lr;
        const bool ok = p < HW;
        const bf16x8 (&dyf)[KS] = dyr[vt];
        // q, k, v (rows d/e = t*16 + 4g + r, column pixel lr) and do
        float qv[2][4], kv[2][4], vv[2][4], dov[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          f32x4 aq = z4, ak = z4, av = z4, ao = z4;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            aq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[0][t][ks], xf[vt][ks], aq, 0, 0, 0);
            ak = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[1][t][ks], xf[vt][ks], ak, 0, 0, 0);
            av = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[2][t][ks], xf[vt][ks], av, 0, 0, 0);
            ao = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[3][t][ks], dyf[ks], ao, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) { qv[t][r] = aq[r]; kv[t][r] = ak[r]; vv[t][r] = av[r]; dov[t][r] = ao[r]; }
        }
        // sm = softmax_d(q); q~ = scale sm
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, qv[t][r]);
        mx = grp4_max(mx);
        float ssum = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            qv[t][r] = __builtin_amdgcn_exp2f((qv[t][r] - mx) * LOG2E);
            ssum += qv[t][r];
          }
        const float inv = __builtin_amdgcn_rcpf(grp4_sum(ssum));
        float qs[2][4], kt[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            qv[t][r] *= inv;              // sm
            qs[t][r] = qv[t][r] * scale;  // q~
            kt[t][r] = __builtin_amdgcn_exp2f(fmaf(kv[t][r], LOG2E, -Kofs[t][r]));  // k~
          }
        const bf16x8 qb = pack_kslot(qs[0], qs[1]);
        const bf16x8 kb = pack_kslot(kt[0], kt[1]);
        const bf16x8 vb = pack_kslot(vv[0], vv[1]);
        const bf16x8 dob = pack_kslot(dov[0], dov[1]);
        float dq[2][4], dk[2][4], dvv[2][4];
        float sdq = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const f32x4 oT = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aT[t], qb, z4, 0, 0, 0);
          const f32x4 dqt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[t], dob, z4, 0, 0, 0);
          const f32x4 dkt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad[t], vb, z4, 0, 0, 0);
          const f32x4 dvt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(adT[t], kb, z4, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dq[t][r] = dqt[r];
            sdq = fmaf(qv[t][r], dqt[r], sdq);
            dk[t][r] = kt[t][r] * (dkt[r] - Gd[t][r]);
            dvv[t][r] = dvt[r];
          }
          if (ok && o_out) {
            float o4[4] = {oT[0], oT[1], oT[2], oT[3]};
            store4(o_out + (rb + p) * INNER + h * DH + t * 16 + lg * 4, o4);
          }
        }
        sdq = grp4_sum(sdq);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) dq[t][r] = scale * qv[t][r] * (dq[t][r] - sdq);
        // stage dq | dk | dv of this pixel tile: row = pixel, column kind*32 + d
        bf16* row = sq + (vt * 16 + lr) * DQLD;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          store4(row + t * 16 + lg * 4, dq[t]);
          store4(row + 32 + t * 16 + lg * 4, dk[t]);
          store4(row + 64 + t * 16 + lg * 4, dvv[t]);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // dxn^T += W_qkv[h rows]^T [dq|dk|dv]^T ; emit dqkv
#pragma unroll
      for (int kind = 0; kind < 3; ++kind) {
        bf16x8 bq[NV];
#pragma unroll
        for (int vt = 0; vt < NV; ++vt) bq[vt] = ld16(sq + (vt * 16 + lr) * DQLD + kind * 32 + lg * 8);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const bf16x8 a = ld_img(wqkv_t, ct, QKV / 32, kind * 8 + h, lane);
#pragma unroll
          for (int vt = 0; vt < NV; ++vt) dxacc[ct][vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq[vt], dxacc[ct][vt], 0, 0, 0);
        }
        if (dqkv_out) {
#pragma unroll
          for (int vt = 0; vt < NV; ++vt) {
            const int p = p0 + vt * 16 + lr;
            if (p < HW) *reinterpret_cast<bf16x8*>(dqkv_out + (rb + p) * QKV + kind * INNER + h * DH + lg * 8) = bq[vt];
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // LN backward + residual; dgamma partial
    if constexpr (C >= 128) {  // (C = 64, NV = 2: 3 more spills)
    // every x / dy load before the first dx store, the stores branch-free through a buffer resource over frame n
    // (pixels past HW go to an out-of-range offset, which the hardware drops): vmcnt retires in issue order, so a
    // load behind a store waits for it -- the per-channel-tile dy load -> dx store rounds serialised CT - 1 store
    // round trips per tile
    {
      const __amdgpu_buffer_rsrc_t drs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(dx + rb * C), (short)0, HW * C * 2, 0x00020000);
      bf16x4 xr[NV][CT], dr[NV][CT];
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) {
        const int p = p0 + vt * 16 + lr;
        const int64_t row = rb + (p < HW ? p : 0);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          xr[vt][ct] = *reinterpret_cast<const bf16x4*>(x + row * C + ct * 16 + lg * 4);
          dr[vt][ct] = *reinterpret_cast<const bf16x4*>(dy + row * C + ct * 16 + lg * 4);
        }
      }
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) {
        const int p = p0 + vt * 16 + lr;
        const bool ok = p < HW;
        float s1 = 0.f, s2 = 0.f;
        float xh[CT][4];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int co = ct * 16 + lg * 4;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            xh[ct][r] = ok ? ((float)xr[vt][ct][r] - mean[vt]) * rstd[vt] : 0.f;
            const float g = dxacc[ct][vt][r] * sgm[co + r];
            s1 += g;
            s2 = fmaf(g, xh[ct][r], s2);
          }
        }
        s1 = grp4_sum(s1) / C;
        s2 = grp4_sum(s2) / C;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int co = ct * 16 + lg * 4;
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
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            o[r] = (bf16)(rstd[vt] * (dxacc[ct][vt][r] * sgm[co + r] - s1 - xh[ct][r] * s2) + (float)dr[vt][ct][r]);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(sl_u32x2, o), drs, ok ? (p * C + co) * 2 : 0x7ffffff0,
                                                0, 0);
        }
      }
    }
    } else {
#pragma unroll
    for (int vt = 0; vt < NV; ++vt) {
      const int p = p0 + vt * 16 + lr;
      const bool ok = p < HW;
      float s1 = 0.f, s2 = 0.f;
      float xh[CT][4];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int co = ct * 16 + lg * 4;
        float xv[4];
        load4(x + (rb + (ok ? p : 0)) * C + co, xv);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xh[ct][r] = ok ? (xv[r] - mean[vt]) * rstd[vt] : 0.f;
          const float g = dxacc[ct][vt][r] * sgm[co + r];
          s1 += g;
          s2 = fmaf(g, xh[ct][r], s2);
        }
      }
      s1 = grp4_sum(s1) / C;
      s2 = grp4_sum(s2) / C;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int co = ct * 16 + lg * 4;
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
        float dv4[4];
        load4(dy + (rb + (ok ? p : 0)) * C + co, dv4);
        if (ok) {
          float o4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o4[r] = rstd[vt] * (dxacc[ct][vt][r] * sgm[co + r] - s1 - xh[ct][r] * s2) + dv4[r];
          store4(dx + (rb + p) * C + co, o4);
        }
      }
    }
    }
  }
  __syncthreads();
  for (int e = tid; e < C; e += 256)
    dgamma_part[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * C + e] =
        ((smem[C + e] + smem[2 * C + e]) + smem[3 * C + e]) + smem[4 * C + e];
}

__global__ __launch_bounds__(256) void slaf_sum_rows_kernel(const float* __restrict__ part, float* __restrict__ dst,
                                                            int nrows, int C, int accumulate) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < nrows; k += 256) s += part[(int64_t)k * C + c];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    s = ((red[0] + red[1]) + red[2]) + red[3];
    dst[c] = accumulate ? dst[c] + s : s;
  }
}

__device__ __forceinline__ void wave_lds_sync_s() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ===================================================================================================
// Head-parallel SLA backward with in-kernel weight gradients (C = 64; the forward ran with LN gamma
// folded into the QKV weights, W' = W diag(gamma), and unit LN gamma).  A block of 8 waves (wave = head)
// takes 48 pixels of one frame at a time: LN (xhat and dy tiles in LDS, block-cooperative) -> per wave:
// raw q|k|v|do of its head (GEMMs) -> per-pixel softmax backward (as slab_dx) -> dq|dk|dv in its LDS slice
// -> dW'_h += dqkv_h^T xhat (register accumulators for the whole kernel) and dxn'_h (this head's share) ->
// the 8 shares summed through LDS -> LN backward -> dx.  No per-voxel intermediate reaches HBM (slab_dx
// emitted the 768-channel dqkv and xn for a separate weight-gradient GEMM).
// ===================================================================================================
// Measured and removed (round 5, profiles/r5f_prefetch_pos_tb.txt, r5f_slah_pb_early_tb.txt, r5_dxt_tb.txt, r5_prio_ab.txt):
// phase B's operands loaded during phase A (+1 %), the dx stores deferred into the next group (10 spills, +5 %), dxn by
// whole output tiles after a block barrier (4.69 -> 5.15 ms per call), s_setprio for waves 4-7 (within the spread);
// round 2: weight fragments without the one-step-ahead pipeline +4 %.
// xhat / dy tiles: region tiles (common.h xt_rs); fp32 partial dxn rows: pl_off layout over the wave's slice
constexpr int SH_SLD = 128;  // slice row stride (bf16): raw q|k|v|do (128 cols), then dq|dk|dv; fp32 partials over it
// Slice layout (round 3): a region tile (common.h rg_off<2>) of eight [R][16] regions -- q, k, v, do, two head-dim
// halves each -- with the two 16-B chunks of a row swapped when bit 2 ^ bit 3 of the row is set: the per-pixel 8-B
// reads of phase B and the transposed dW reads are conflict-free, the dxn fragment reads 2-way, the column stores
// 2-way (the minimum); each access site needs one per-lane offset register (tools/lds_banks.py).  Round 2's 272-B
// rows were 2-way on the fragment and transposed reads (42 % of slah_dx's LDS cycles were conflicts).
template <int R>
__device__ __forceinline__ int sl_off(int r, int c) { return rg_off<2>(r, c, R * 16); }

static size_t slah_smem(int NV) {
  const int R = 16 * NV;
  return (size_t)2 * xt_elems(R) * 2 + (size_t)8 * R * SH_SLD * 2;
}

template <int NV>
__global__ __launch_bounds__(512, 1) void slah_dx_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, const bf16* __restrict__ wqkv,
    const bf16* __restrict__ wqkv_t, const bf16* __restrict__ wout_t, const float* __restrict__ kimg,
    const bf16* __restrict__ actT, const bf16* __restrict__ actx, const bf16* __restrict__ adc,
    const bf16* __restrict__ adcT, bf16* __restrict__ dx, float* __restrict__ dw_slab, int Nf, int HW, float scale,
    float eps) {
  constexpr int C = 64, KS = C / 32, CT = C / 16, R = 16 * NV;
  static_assert(TH_PLD * 4 <= SH_SLD * 2, "partial dxn rows fit over the slice rows");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  bf16* xt = reinterpret_cast<bf16*>(smem);  // [R][64] xhat (region tile, xt_rs)
  bf16* dyt = xt + xt_elems(R);               // [R][64] dy
  bf16* slices = dyt + xt_elems(R);           // 8 x [R][SH_SLD] (sl_off layout)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int h = wid;
  bf16* sl = slices + wid * R * SH_SLD;
  const int npg = (HW + R - 1) / R;
  const int ngroups = Nf * npg;
  const int vv = tid >> 3, cc = tid & 7;  // LN role: pixel vv of the group, channels 8cc..8cc+7
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};

  auto prow = [&](int gg) -> int64_t {  // row of this thread's pixel in group gg, or -1
    if (gg >= ngroups || vv >= R) return -1;
    const int n = gg / npg, p = (gg - n * npg) * R + vv;
    return p < HW ? (int64_t)n * HW + p : -1;
  };
  bf16x8 xpf = zero8(), dpf = zero8();
  bool okpf = false;
  auto prefetch = [&](int gg) {
    const int64_t row = prow(gg);
    okpf = row >= 0;
    const int64_t rr = okpf ? row : 0;
    xpf = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(x + rr * C + cc * 8));
    dpf = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(dy + rr * C + cc * 8));
  };

  f32x4 dwacc[6][4];
#pragma unroll
  for (int m = 0; m < 6; ++m)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dwacc[m][nt] = z4;

  prefetch(blockIdx.x);
  for (int gg = blockIdx.x; gg < ngroups; gg += gridDim.x) {
    const int n = gg / npg, p0 = (gg - n * npg) * R;
    // ---- LN of this thread's pixel chunk (statistics over its 8 lanes)
    const bool ok_cur = okpf;
    float rstd_cur;
    {
      float a[8], s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) { a[e] = ok_cur ? (float)xpf[e] : 0.f; s += a[e]; }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) s += __shfl_xor(s, o, 64);
      const float mean = s * (1.f / C);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = a[e] - mean; q = fmaf(d, d, q); }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) q += __shfl_xor(q, o, 64);
      const float rstd = 1.f / sqrtf(q * (1.f / C) + eps);
      rstd_cur = ok_cur ? rstd : 0.f;
      if (vv < R) {
        bf16x8 xh, dv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[e] = (bf16)(ok_cur ? (a[e] - mean) * rstd : 0.f);
          dv[e] = ok_cur ? dpf[e] : (bf16)0.f;
        }
        *reinterpret_cast<bf16x8*>(xt + rg_off<1>(vv, cc * 8, xt_rs(R))) = xh;
        *reinterpret_cast<bf16x8*>(dyt + rg_off<1>(vv, cc * 8, xt_rs(R))) = dv;
      }
    }
    const int oz = opaque_zero();
    const bf16* wq_g = wqkv + oz;
    const bf16* wqt_g = wqkv_t + oz;
    const bf16* wot_g = wout_t + oz;
    // phase A's weight fragments double-buffered per kind: kind 0 issued before barrier A (its L2 latency
    // overlaps the barrier wait), kind k+1 before kind k's MFMAs
    bf16x8 wa[2][2][KS];
    auto lda = [&](int kind, int buf) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          wa[buf][t][ks] = kind < 3 ? ld_img(wq_g, kind * 16 + h * 2 + t, KS, ks, lane) : ld_img(wot_g, h * 2 + t, KS, ks, lane);
    };
    lda(0, 0);
    __syncthreads();  // (A)

    // phase B's per-(frame, head) operands (L2-resident images)
    bf16x8 aT[2], ax[2], ad[2], adT[2];
    f32x4 kg[4];
    auto ldpb = [&]() {
      const int64_t fo = ((int64_t)(n * NH + h) * 2) * 64 * 8;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        aT[t] = ld16(actT + fo + (t * 64 + lane) * 8);
        ax[t] = ld16(actx + fo + (t * 64 + lane) * 8);
        ad[t] = ld16(adc + fo + (t * 64 + lane) * 8);
        adT[t] = ld16(adcT + fo + (t * 64 + lane) * 8);
      }
      const f32x4* ki = reinterpret_cast<const f32x4*>(kimg + ((int64_t)(n * NH + h) * 64 + lane) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) kg[q] = ki[q];
      // the next group's x / dy behind phase A's weights and these operands (vmcnt retires in issue order: a load
      // issued behind the HBM prefetch waits for it; round 5, issued after barrier A: +3.5 %)
      prefetch(gg + gridDim.x);
    };

    // ---- phase A: raw q | k | v | do of head h, rows = pixels, cols kind*32 + d
#pragma unroll
    for (int kind = 0; kind < 4; ++kind) {
      if (kind + 1 < 4) lda(kind + 1, (kind + 1) & 1);
      const auto& a = wa[kind & 1];
      const bf16* src = kind < 3 ? xt : dyt;
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) {
        bf16x8 b[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) b[ks] = ld16(src + rg_off<1>(vt * 16 + lr, ks * 32 + lg * 8, xt_rs(R)));
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          f32x4 acc = z4;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][ks], b[ks], acc, 0, 0, 0);
          float o4[4] = {acc[0], acc[1], acc[2], acc[3]};
          store4(sl + sl_off<R>(vt * 16 + lr, kind * 32 + t * 16 + lg * 4), o4);
        }
      }
    }
    wave_lds_sync_s();
    // ---- phase B: per-pixel softmax backward (slab_dx's math); dq | dk | dv over cols 0..95
    {
      ldpb();
      float Kofs[2][4], Gd[2][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { Kofs[0][r] = kg[0][r]; Kofs[1][r] = kg[1][r]; Gd[0][r] = kg[2][r]; Gd[1][r] = kg[3][r]; }
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) {
        const bool ok = p0 + vt * 16 + lr < HW;
        const int rw = vt * 16 + lr;
        float qv[2][4], kv[2][4], vv4[2][4], dov[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          load4(sl + sl_off<R>(rw, 0 * 32 + t * 16 + lg * 4), qv[t]);
          load4(sl + sl_off<R>(rw, 1 * 32 + t * 16 + lg * 4), kv[t]);
          load4(sl + sl_off<R>(rw, 2 * 32 + t * 16 + lg * 4), vv4[t]);
          load4(sl + sl_off<R>(rw, 3 * 32 + t * 16 + lg * 4), dov[t]);
        }
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, qv[t][r]);
        mx = grp4_max(mx);
        float ssum = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            qv[t][r] = __builtin_amdgcn_exp2f((qv[t][r] - mx) * LOG2E);
            ssum += qv[t][r];
          }
        const float inv = __builtin_amdgcn_rcpf(grp4_sum(ssum));
        float qs[2][4], kt[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            qv[t][r] *= inv;
            qs[t][r] = qv[t][r] * scale;
            kt[t][r] = __builtin_amdgcn_exp2f(fmaf(kv[t][r], LOG2E, -Kofs[t][r]));
          }
        const bf16x8 qb = pack_kslot(qs[0], qs[1]);
        const bf16x8 kb = pack_kslot(kt[0], kt[1]);
        const bf16x8 vb = pack_kslot(vv4[0], vv4[1]);
        const bf16x8 dob = pack_kslot(dov[0], dov[1]);
        float dq[2][4], dk[2][4], dvv[2][4];
        float sdq = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const f32x4 dqt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[t], dob, z4, 0, 0, 0);
          const f32x4 dkt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad[t], vb, z4, 0, 0, 0);
          const f32x4 dvt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(adT[t], kb, z4, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dq[t][r] = dqt[r];
            sdq = fmaf(qv[t][r], dqt[r], sdq);
            dk[t][r] = kt[t][r] * (dkt[r] - Gd[t][r]);
            dvv[t][r] = dvt[r];
          }
        }
        (void)qb;
        sdq = grp4_sum(sdq);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dq[t][r] = ok ? scale * qv[t][r] * (dq[t][r] - sdq) : 0.f;
            dk[t][r] = ok ? dk[t][r] : 0.f;
            dvv[t][r] = ok ? dvv[t][r] : 0.f;
          }
        // each lane overwrites exactly the q / k / v entries it read itself: no sync needed
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          store4(sl + sl_off<R>(rw, t * 16 + lg * 4), dq[t]);
          store4(sl + sl_off<R>(rw, 32 + t * 16 + lg * 4), dk[t]);
          store4(sl + sl_off<R>(rw, 64 + t * 16 + lg * 4), dvv[t]);
        }
      }
    }
    wave_lds_sync_s();
    // the dxn GEMM's W'^T fragments one ahead: the first in flight during the dW GEMM
    bf16x8 wring[2];
    auto ldw = [&](int idx) { return ld_img(wqt_g, idx % CT, QKV / 32, (idx / CT) * 8 + h, lane); };
    wring[0] = ldw(0);
    // ---- dW'_h += dqkv_h^T . xhat (K = pixels, 16 per step)
#pragma unroll
    for (int kk = 0; kk < NV; ++kk) {
      s16x4 bx[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bx[nt] = tr4_rg<1>(xt, kk * 16, nt * 16, xt_rs(R), lane);
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        const s16x4 a = tr4_rg<2>(sl, kk * 16, (m >> 1) * 32 + (m & 1) * 16, R * 16, lane);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          dwacc[m][nt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bx[nt], dwacc[m][nt], 0, 0, 0);
      }
    }
    // ---- dxn'_h (this head's share of g = gamma * dxn)
    f32x4 dxacc[CT][NV];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int vt = 0; vt < NV; ++vt) dxacc[ct][vt] = z4;
#pragma unroll
    for (int kind = 0; kind < 3; ++kind)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int idx = kind * CT + ct;
        if (idx + 1 < 3 * CT) wring[(idx + 1) & 1] = ldw(idx + 1);
        const bf16x8 a = wring[idx & 1];
#pragma unroll
        for (int vt = 0; vt < NV; ++vt)
          dxacc[ct][vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ld16(sl + sl_off<R>(vt * 16 + lr, kind * 32 + lg * 8)),
                                                                  dxacc[ct][vt], 0, 0, 0);
      }
    wave_lds_sync_s();
    {
      float* part = reinterpret_cast<float*>(sl);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int vt = 0; vt < NV; ++vt)
          *reinterpret_cast<f32x4*>(part + pl_off(vt * 16 + lr, ct * 16 + lg * 4)) = dxacc[ct][vt];
    }
    __syncthreads();  // (B)
    // ---- LN backward of this thread's pixel chunk
    {
      const int v = vv < R ? vv : 0;
      float g[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        const float* pw = reinterpret_cast<const float*>(slices + w * R * SH_SLD);
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(pw + pl_off(v, cc * 8));
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(pw + pl_off(v, cc * 8 + 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) { g[e] += a0[e]; g[4 + e] += a1[e]; }
      }
      const bf16x8 xh = *reinterpret_cast<const bf16x8*>(xt + rg_off<1>(v, cc * 8, xt_rs(R)));
      const bf16x8 dv = *reinterpret_cast<const bf16x8*>(dyt + rg_off<1>(v, cc * 8, xt_rs(R)));
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1 += g[e]; s2 = fmaf(g[e], (float)xh[e], s2); }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
      s1 *= 1.f / C;
      s2 *= 1.f / C;
      if (vv < R && ok_cur) {
        bf16x8 o8;
#pragma unroll
        for (int e = 0; e < 8; ++e) o8[e] = (bf16)(rstd_cur * (g[e] - s1 - (float)xh[e] * s2) + (float)dv[e]);
        __builtin_nontemporal_store(o8, reinterpret_cast<bf16x8*>(dx + ((int64_t)n * HW + p0 + vv) * C + cc * 8));
      }
    }
  }
  float* slab = dw_slab + (int64_t)blockIdx.x * QKV * C;
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const int j0 = (m >> 1) * INNER + h * DH + (m & 1) * 16 + lg * 4;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(int64_t)(j0 + r) * C + nt * 16 + lr] = dwacc[m][nt][r];
  }
}

__global__ void pack_scaled_kernel(const float* __restrict__ w, const float* __restrict__ cs, bf16* __restrict__ out,
                                   int M, int K, int trans) {
  const int64_t n = (int64_t)M * K;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int m = (int)(e / K), k = (int)(e - (int64_t)m * K);
    const bf16 v = (bf16)(w[e] * (cs ? cs[k] : 1.f));
    if (trans) out[(int64_t)k * M + m] = v;
    else out[e] = v;
  }
}

}  // namespace

extern "C" {

// blocks per frame used by the stats / dctx kernels (each covers spb 64-pixel sub-chunks)
int cesm_slaf_nblk(int Nf, int HW) {
  const int nsc = (HW + 63) / 64;
  int nblk = std::min(std::max(1, 1024 / std::max(1, Nf)), SLAF_NBLK_MAX);  // combine reduces <= 128 partials
  nblk = std::min(nblk, nsc);
  const int spb = (nsc + nblk - 1) / nblk;
  return (nsc + spb - 1) / spb;
}

// Fused SLA block forward (bf16, C = 64).  x, y [Nf*HW][C]; wqkv [768][C], wout [C][256] packed bf16;
// saved for the backward: mz [Nf][8][32][2] (softmax max / normaliser of k over pixels),
// ctx32 [Nf][8][32][32] fp32, actT / actx [Nf][8][2][64][8] bf16 (ctx as MFMA A fragments).
// ws: cesm_slaf_nblk(Nf, HW) * Nf * 8 * 1088 floats.
int cesm_slaf_fwd(const void* x, const float* gamma, const void* wqkv, const void* wout, const float* bout, void* y,
                  void* o, float* mz, float* ctx32, void* actT, void* actx, float* ws, int Nf, int HW, int C,
                  float scale, float eps, hipStream_t stream) {
  if ((C != 64 && C != 128) || Nf < 1 || HW < 1) return CESM_EUNSUPPORTED;
  const int nsc = (HW + 63) / 64;
  const int nblk = cesm_slaf_nblk(Nf, HW);
  const int spb = (nsc + nblk - 1) / nblk;
  if (C == 64)
    slaf_stats_kernel<64><<<dim3(nblk, Nf), 512, 0, stream>>>((const bf16*)x, gamma, (const bf16*)wqkv, ws, HW, spb, eps);
  else
    slaf_stats_kernel<128><<<dim3(nblk, Nf), 512, 0, stream>>>((const bf16*)x, gamma, (const bf16*)wqkv, ws, HW, spb, eps);
  slaf_combine_kernel<<<Nf * NH, 256, 0, stream>>>(ws, nblk, mz, ctx32, (bf16*)actT, (bf16*)actx);
  if (C == 64)
    slaf_out_kernel<64, 4><<<dim3((unsigned)cdiv(HW, 64 * 4), Nf), 256, 0, stream>>>(
        (const bf16*)x, gamma, (const bf16*)wqkv, (const bf16*)wout, bout, (const bf16*)actT, (bf16*)y, (bf16*)o, HW, scale, eps);
  else
    slaf_out_kernel<128, 2><<<dim3((unsigned)cdiv(HW, 64 * 2), Nf), 256, 0, stream>>>(
        (const bf16*)x, gamma, (const bf16*)wqkv, (const bf16*)wout, bout, (const bf16*)actT, (bf16*)y, (bf16*)o, HW, scale, eps);
  return cesm_launch_status();
}

// Fused SLA block backward (bf16, C = 64), dx path: dx (+ dy residual), dgamma (+)=, and for the weight
// gradients dqkv [Nf*HW][768], o [Nf*HW][256], xn [Nf*HW][C] (each nullable).  mz/ctx32/actT/actx from
// cesm_slaf_fwd; wqkv_t [C][768] and wout_t [256][C] swap-packed.  ws: max(nblk*Nf*8*1024, ...) floats
// + Nf*8*(32 + 2*2*64*8/2) + grid*C (see kernels.slaf_bwd for the carve-up).
int cesm_slaf_bwd(const void* x, const void* dy, const float* gamma, const void* wqkv, const void* wqkv_t,
                  const void* wout_t, const float* mz, const float* ctx32, const void* actT, const void* actx,
                  void* dx, void* dqkv, void* o, void* xn, float* dgamma, float* part, float* G, void* adc, void* adcT,
                  float* dgp, void* wimg, int Nf, int HW, int C, float scale, float eps, int accumulate,
                  hipStream_t stream) {
  if ((C != 64 && C != 128) || Nf < 1 || HW < 1) return CESM_EUNSUPPORTED;
  // fragment images of W_qkv [768][C], W_qkv^T [C][768], W_out^T [256][C] for slab_dx
  bf16* img_q = (bf16*)wimg;
  bf16* img_qt = img_q + 768 * C;
  bf16* img_ot = img_qt + 768 * C;
  frag_image(wqkv, img_q, 768, C, stream);
  frag_image(wqkv_t, img_qt, C, 768, stream);
  frag_image(wout_t, img_ot, 256, C, stream);
  const int nsc = (HW + 63) / 64;
  const int nblk = cesm_slaf_nblk(Nf, HW);
  const int spb = (nsc + nblk - 1) / nblk;
  if (C == 64)
    slab_dctx_kernel<64><<<dim3(nblk, Nf), 512, 0, stream>>>((const bf16*)x, (const bf16*)dy, gamma, (const bf16*)wqkv,
                                                             (const bf16*)wout_t, part, HW, spb, scale, eps);
  else
    slab_dctx_kernel<128><<<dim3(nblk, Nf), 512, 0, stream>>>((const bf16*)x, (const bf16*)dy, gamma,
                                                              (const bf16*)wqkv, (const bf16*)wout_t, part, HW, spb,
                                                              scale, eps);
  slab_combine_kernel<<<Nf * NH, 256, 0, stream>>>(part, nblk, ctx32, mz, G, (bf16*)adc, (bf16*)adcT);
  // NV = 16-pixel tiles per wave: 2 at C = 64, 1 at C = 128 (registers); dgp rows = grid blocks
  const int NVr = C == 64 ? 2 : 1;
  dim3 grid((unsigned)cdiv(HW, 64 * NVr), Nf);
  const size_t sm = (size_t)C * 20 + (size_t)4 * 16 * NVr * DQLD * 2;
  if (C == 64)
    slab_dx_kernel<64, 2><<<grid, 256, sm, stream>>>(
        (const bf16*)x, (const bf16*)dy, gamma, img_q, img_qt, img_ot, G,
        (const bf16*)actT, (const bf16*)actx, (const bf16*)adc, (const bf16*)adcT, (bf16*)dx, (bf16*)dqkv, (bf16*)o,
        (bf16*)xn, dgp, HW, scale, eps);
  else
    slab_dx_kernel<128, 1><<<grid, 256, sm, stream>>>(
        (const bf16*)x, (const bf16*)dy, gamma, img_q, img_qt, img_ot, G,
        (const bf16*)actT, (const bf16*)actx, (const bf16*)adc, (const bf16*)adcT, (bf16*)dx, (bf16*)dqkv, (bf16*)o,
        (bf16*)xn, dgp, HW, scale, eps);
  if (dgamma) slaf_sum_rows_kernel<<<C, 256, 0, stream>>>(dgp, dgamma, (int)(grid.x * grid.y), C, accumulate);
  return cesm_launch_status();
}

// grid blocks of cesm_slaf_bwd's dx kernel (rows of its dgamma partial)
int cesm_slaf_bwd_nblk(int Nf, int HW, int C) { return (int)cdiv(HW, C == 64 ? 128 : 64) * Nf; }

// blocks of cesm_slaf_bwd_dw's head-parallel dx kernel (one per CU); 0 = shape not supported
int cesm_slaf_bwd_dw_nblk(int Nf, int HW, int C) {
  if (C != 64 || Nf < 1 || HW < 1) return 0;
  const int ngroups = Nf * (int)cdiv(HW, 48);
  return std::min(ngroups, cesm_num_cus());
}

// Fused SLA block backward with in-kernel weight gradients (C = 64).  The forward (cesm_slaf_fwd) must have
// run with gamma_one (unit LN gamma) and wq_fold = bf16 W diag(gamma) [768][C] (cesm_pack_scaled); the same
// two go to the dctx pass here.  dx; dwqkv (+)= dW_qkv and dgamma (+)= the LN gamma gradient (nullable).
// Workspaces as cesm_slaf_bwd for part / G / adc / adcT; slab nblk_dx*768*C and tmp 768*C floats;
// wimg (2*768 + 256)*C bf16.
int cesm_slaf_bwd_dw(const void* x, const void* dy, const float* gamma_one, const void* wq_fold, const float* wqkv_f32,
                     const float* gamma, const void* wout_t, const float* mz, const float* ctx32, const void* actT,
                     const void* actx, void* dx, float* dwqkv, float* dgamma, float* dwout, float* dbout, float* part,
                     float* G, void* adc, void* adcT, float* slab, float* tmp, float* partm, float* partb, void* wimg,
                     int nblk_dx, int Nf, int HW, int C, float scale, float eps, int accumulate, hipStream_t stream) {
  if (nblk_dx < 1 || nblk_dx != cesm_slaf_bwd_dw_nblk(Nf, HW, C)) return CESM_EUNSUPPORTED;
  const bool dwo = dwout || dbout;
  if (dwo && (!partm || !partb || !dwout || !dbout)) return CESM_EINVAL;
  bf16* img_q = (bf16*)wimg;
  bf16* img_qt = img_q + 768 * C;
  bf16* img_ot = img_qt + 768 * C;
  frag_image(wq_fold, img_q, 768, C, stream);
  frag_image_f32_kernel<<<(unsigned)cdiv((int64_t)768 * C / 8, 256), 256, 0, stream>>>(wqkv_f32, gamma, img_qt, C,
                                                                                          768, 1);
  frag_image(wout_t, img_ot, 256, C, stream);
  const int nsc = (HW + 63) / 64;
  const int nblk = cesm_slaf_nblk(Nf, HW);
  const int spb = (nsc + nblk - 1) / nblk;
  if (dwo) {
    slab_dctx_kernel<64, true><<<dim3(nblk, Nf), 512, 0, stream>>>((const bf16*)x, (const bf16*)dy, gamma_one,
                                                                   (const bf16*)wq_fold, (const bf16*)wout_t, part, HW,
                                                                   spb, scale, eps, partm, partb);
    // partm is re-used for R once the per-frame products are formed (R: Nf*8*2048 floats <= partm)
    float* R = partm + (int64_t)Nf * nblk * NH * 2048;
    slab_dwout_frame_kernel<<<Nf * NH, 256, 0, stream>>>(partm, nblk, ctx32, R);
    slab_dwout_sum_kernel<<<64, 256, 0, stream>>>(R, Nf, dwout, accumulate);
    slaf_sum_rows_kernel<<<64, 256, 0, stream>>>(partb, dbout, Nf * nblk, 64, accumulate);
  } else {
    slab_dctx_kernel<64><<<dim3(nblk, Nf), 512, 0, stream>>>((const bf16*)x, (const bf16*)dy, gamma_one,
                                                             (const bf16*)wq_fold, (const bf16*)wout_t, part, HW, spb,
                                                             scale, eps);
  }
  slab_combine_kernel<<<Nf * NH, 256, 0, stream>>>(part, nblk, ctx32, mz, G, (bf16*)adc, (bf16*)adcT);
  const size_t sm = slah_smem(3);
  (void)hipFuncSetAttribute((const void*)slah_dx_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  slah_dx_kernel<3><<<nblk_dx, 512, sm, stream>>>((const bf16*)x, (const bf16*)dy, img_q, img_qt, img_ot, G,
                                                  (const bf16*)actT, (const bf16*)actx, (const bf16*)adc,
                                                  (const bf16*)adcT, (bf16*)dx, slab, Nf, HW, scale, eps);
  const int64_t nel = (int64_t)768 * C;
  twh_dw_reduce_kernel<<<twh_dw_reduce_grid(nel), 256, 0, stream>>>(slab, nblk_dx, wqkv_f32, gamma, dwqkv, tmp, 768,
                                                                    C, accumulate);
  if (dgamma) twh_dgamma_kernel<<<C, 256, 0, stream>>>(tmp, dgamma, 768, C, accumulate);
  return cesm_launch_status();
}

// out[m][k] = bf16(w[m][k] * colscale[k]), w fp32 row-major [M][K] (trans = 0); trans = 1: out [K][M] = its
// transpose (the swap-packed layout)
int cesm_pack_scaled(const float* w, const float* colscale, void* out, int M, int K, int trans, hipStream_t stream) {
  if (M < 1 || K < 1) return CESM_EINVAL;
  const int64_t n = (int64_t)M * K;
  pack_scaled_kernel<<<(unsigned)std::min<int64_t>(cdiv(n, 256), 4096), 256, 0, stream>>>(w, colscale, (bf16*)out, M,
                                                                                          K, trans);
  return cesm_launch_status();
}

}  // extern "C"
