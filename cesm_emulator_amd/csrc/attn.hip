// Attention cores of video_net:
//  * temporal softmax attention (video_net.py:368-454): per pixel, per head, over the frame
//    axis F: q*scale -> RoPE (rotary_embedding.py:29-48, 146-163) on q and k -> q.k + rel-pos
//    bias (video_net.py:268-310) -> softmax -> attn.v.  The QKV / output projections run on the
//    MFMA conv kernel as 1x1 convs; this file is the per-pixel core (tiny F x F x 32 problems,
//    VALU, one lane per (pixel, head, frame); each lane rotates only its own q/k row and shares
//    it with the other F lanes of its pixel through LDS).
//  * spatial linear attention core (video_net.py:313-347): k-softmax over all H*W positions of
//    a frame (split-n with rescaled partial contexts, deterministic combine), q-softmax over the
//    32 head dims, out = context^T q (one head per wave: the context is an LDS broadcast).
//
// Layouts (channels-last, voxel v = (b*F + f)*HW + p):
//   qkv [V][768] = q | k | v, head-major inside each (channel = h*32 + d)
//   out [V][256]
#include "common.h"
#include "cesm_hip.h"

namespace {

constexpr int DH = 32;      // head dim
constexpr int NH = 8;       // heads
constexpr int INNER = 256;  // NH*DH
constexpr int QKV = 768;
constexpr int TA_T = 128;   // threads per temporal-attention block
constexpr int TA_LD = 36;   // padded LDS row (floats) for a staged 32-vector

// rot[f][i] = (cos, sin) of f * freqs[i], i < 16
__global__ void rope_table_kernel(const float* __restrict__ freqs, float* __restrict__ rot, int F) {
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  if (t >= F * 16) return;
  const int f = t / 16, i = t % 16;
  const float a = (float)f * freqs[i];
  rot[t * 2] = cosf(a);
  rot[t * 2 + 1] = sinf(a);
}

template <typename T>
__device__ __forceinline__ void load32(const T* p, float* v) {
#pragma unroll
  for (int i = 0; i < 32; i += 8) load8(p + i, v + i);
}
template <typename T>
__device__ __forceinline__ void store32(T* p, const float* v) {
#pragma unroll
  for (int i = 0; i < 32; i += 8) store8(p + i, v + i);
}
__device__ __forceinline__ void lds_store32(float* p, const float* v) {
#pragma unroll
  for (int i = 0; i < 32; i += 4) *reinterpret_cast<f32x4*>(p + i) = f32x4{v[i], v[i + 1], v[i + 2], v[i + 3]};
}
__device__ __forceinline__ void lds_load32(const float* p, float* v) {
#pragma unroll
  for (int i = 0; i < 32; i += 4) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p + i);
    v[i] = a[0]; v[i + 1] = a[1]; v[i + 2] = a[2]; v[i + 3] = a[3];
  }
}
// x'[2i] = x[2i] c - x[2i+1] s ; x'[2i+1] = x[2i+1] c + x[2i] s   (sign = +1)
// inverse (transpose) with sign = -1
__device__ __forceinline__ void rope(float* v, const float* rot, float sign) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float c = rot[i * 2], s = sign * rot[i * 2 + 1];
    const float a = v[2 * i], b = v[2 * i + 1];
    v[2 * i] = a * c - b * s;
    v[2 * i + 1] = b * c + a * s;
  }
}

// grid: x = pixel-block (grid-stride), y = b*NH + h.  Block = G = TA_T/F groups of F lanes.
// VLDS (long windows, F > 32): the pixel's v rows are staged in LDS next to k, so the per-key v read is
// an LDS broadcast instead of the same global row loaded by all F lanes
template <typename T, bool VLDS = false>
__global__ __launch_bounds__(TA_T) void tattn_fwd_kernel(const T* __restrict__ qkv, const float* __restrict__ bias,
                                                         const float* __restrict__ rotg, T* __restrict__ out,
                                                         float* __restrict__ lse, int F, int HW, float scale) {
  extern __shared__ __attribute__((aligned(16))) float ta_dyn[];  // tables sized by F (ta_fwd_smem)
  float* rot = ta_dyn;        // [F][32]
  float* sb = rot + F * 32;   // [F][F]
  float* svl = ta_dyn + ((F * 32 + F * F + 3) & ~3);  // VLDS: [TA_T][TA_LD] v rows
  __shared__ __attribute__((aligned(16))) float sk[TA_T * TA_LD];
  const int b = blockIdx.y / NH, h = blockIdx.y % NH;
  for (int e = threadIdx.x; e < F * 32; e += blockDim.x) rot[e] = rotg[e];
  for (int e = threadIdx.x; e < F * F; e += blockDim.x) sb[e] = bias[h * F * F + e];
  __syncthreads();
  const int G = TA_T / F;
  const int g = threadIdx.x / F, i = threadIdx.x % F;
  const bool lane_ok = g < G;
  const int npb = (HW + G - 1) / G;
  for (int pb = blockIdx.x; pb < npb; pb += gridDim.x) {
    const int p = pb * G + g;
    const bool ok = lane_ok && p < HW;
    const int64_t vi = ((int64_t)b * F + i) * HW + p;
    float q[32];
    if (ok) {
      float k[32];
      load32(qkv + vi * QKV + INNER + h * DH, k);
      rope(k, rot + i * 32, 1.f);
      lds_store32(sk + threadIdx.x * TA_LD, k);
      if constexpr (VLDS) {
        float vv[32];
        load32(qkv + vi * QKV + 2 * INNER + h * DH, vv);
        lds_store32(svl + threadIdx.x * TA_LD, vv);
      }
      load32(qkv + vi * QKV + h * DH, q);
#pragma unroll
      for (int d = 0; d < 32; ++d) q[d] *= scale;
      rope(q, rot + i * 32, 1.f);
    }
    __syncthreads();
    if (ok) {
      float acc[32];
#pragma unroll
      for (int d = 0; d < 32; ++d) acc[d] = 0.f;
      float m = -INFINITY, l = 0.f;
      for (int j = 0; j < F; ++j) {
        float k[32], v[32];
        lds_load32(sk + (g * F + j) * TA_LD, k);
        float s = 0.f;
#pragma unroll
        for (int d = 0; d < 32; ++d) s = fmaf(q[d], k[d], s);
        s += sb[i * F + j];
        if constexpr (VLDS) {
          lds_load32(svl + (g * F + j) * TA_LD, v);
        } else {
          const int64_t vj = ((int64_t)b * F + j) * HW + p;
          load32(qkv + vj * QKV + 2 * INNER + h * DH, v);
        }
        const float mn = fmaxf(m, s);
        const float corr = expf(m - mn);
        const float pj = expf(s - mn);
        l = l * corr + pj;
#pragma unroll
        for (int d = 0; d < 32; ++d) acc[d] = fmaf(pj, v[d], acc[d] * corr);
        m = mn;
      }
      const float inv = 1.f / l;
#pragma unroll
      for (int d = 0; d < 32; ++d) acc[d] *= inv;
      store32(out + vi * INNER + h * DH, acc);
      if (lse) lse[(((int64_t)b * NH + h) * HW + p) * F + i] = m + logf(l);
    }
    __syncthreads();
  }
}

// backward.  Phase 1 (lane = query i): D_i, dq_i, dbias row accumulation (k' rows in LDS).
//            Phase 2 (lane = key j):   dk_j, dv_j (q' rows in LDS).
// dbias partials: part[blockIdx.y][blockIdx.x][i][j] (the block's sum over its pixels)
// VLDS (long windows, F > 32): the bias is read from global memory (cached) instead of an [F][F] LDS
// table, and that LDS holds the pixel's v rows (phase 1) / dO rows (phase 2) instead, so the per-key
// row read is an LDS broadcast rather than the same global row loaded by all F lanes
template <typename T, bool VLDS = false>
__global__ __launch_bounds__(TA_T) void tattn_bwd_kernel(const T* __restrict__ qkv, const T* __restrict__ o,
                                                         const T* __restrict__ dout, const float* __restrict__ lse,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ rotg, T* __restrict__ dqkv,
                                                         float* __restrict__ dbias_part, int F, int HW,
                                                         float scale) {
  extern __shared__ __attribute__((aligned(16))) float ta_dyn[];  // tables sized by F (ta_bwd_smem)
  const int AS = F + 1;                 // dbias row stride (odd: conflict-free column walks)
  float* rot = ta_dyn;                  // [F][32]
  float* sb = rot + F * 32;             // [F][F] (VLDS: v / dO rows [TA_T][TA_LD])
  float* sacc = sb + (VLDS ? TA_T * TA_LD : F * F);  // [TA_T][F + 1] per-lane dbias rows
  const float* gbias = bias + (int64_t)(blockIdx.y % NH) * F * F;
  __shared__ __attribute__((aligned(16))) float sv[TA_T * TA_LD];  // k' (phase 1) / q' (phase 2)
  __shared__ float sD[TA_T], sL[TA_T];
  const int b = blockIdx.y / NH, h = blockIdx.y % NH;
  for (int e = threadIdx.x; e < F * 32; e += blockDim.x) rot[e] = rotg[e];
  if constexpr (!VLDS)
    for (int e = threadIdx.x; e < F * F; e += blockDim.x) sb[e] = bias[h * F * F + e];
  for (int e = threadIdx.x; e < TA_T * AS; e += blockDim.x) sacc[e] = 0.f;
  __syncthreads();
  const int G = TA_T / F;
  const int g = threadIdx.x / F, i = threadIdx.x % F;
  const bool lane_ok = g < G;
  float* myacc = sacc + threadIdx.x * AS;
  const int npb = (HW + G - 1) / G;
  for (int pb = blockIdx.x; pb < npb; pb += gridDim.x) {
    const int p = pb * G + g;
    const bool ok = lane_ok && p < HW;
    const int64_t vi = ((int64_t)b * F + i) * HW + p;
    // ---- phase 1: stage k'_i
    float D = 0.f, L = 0.f;
    if (ok) {
      float k[32];
      load32(qkv + vi * QKV + INNER + h * DH, k);
      rope(k, rot + i * 32, 1.f);
      lds_store32(sv + threadIdx.x * TA_LD, k);
      if constexpr (VLDS) {
        float vv[32];
        load32(qkv + vi * QKV + 2 * INNER + h * DH, vv);
        lds_store32(sb + threadIdx.x * TA_LD, vv);
      }
    }
    __syncthreads();
    if (ok) {
      float q[32], dq[32], dO[32];
      load32(dout + vi * INNER + h * DH, dO);
      {
        float ov[32];
        load32(o + vi * INNER + h * DH, ov);
#pragma unroll
        for (int d = 0; d < 32; ++d) D = fmaf(dO[d], ov[d], D);
      }
      L = lse[(((int64_t)b * NH + h) * HW + p) * F + i];
      load32(qkv + vi * QKV + h * DH, q);
#pragma unroll
      for (int d = 0; d < 32; ++d) { q[d] *= scale; dq[d] = 0.f; }
      rope(q, rot + i * 32, 1.f);
      for (int j = 0; j < F; ++j) {
        float k[32], v[32];
        lds_load32(sv + (g * F + j) * TA_LD, k);
        if constexpr (VLDS) {
          lds_load32(sb + (g * F + j) * TA_LD, v);
        } else {
          const int64_t vj = ((int64_t)b * F + j) * HW + p;
          load32(qkv + vj * QKV + 2 * INNER + h * DH, v);
        }
        float s = 0.f, dp = 0.f;
#pragma unroll
        for (int d = 0; d < 32; ++d) { s = fmaf(q[d], k[d], s); dp = fmaf(dO[d], v[d], dp); }
        s += VLDS ? gbias[i * F + j] : sb[i * F + j];
        const float P = expf(s - L);
        const float dS = P * (dp - D);
        myacc[j] += dS;
#pragma unroll
        for (int d = 0; d < 32; ++d) dq[d] = fmaf(dS, k[d], dq[d]);
      }
      rope(dq, rot + i * 32, -1.f);
#pragma unroll
      for (int d = 0; d < 32; ++d) dq[d] *= scale;
      store32(dqkv + vi * QKV + h * DH, dq);
    }
    sD[threadIdx.x] = D;
    sL[threadIdx.x] = L;
    __syncthreads();
    // ---- phase 2: stage q'_i, lane acts as key row j = i
    if (ok) {
      float q[32];
      load32(qkv + vi * QKV + h * DH, q);
#pragma unroll
      for (int d = 0; d < 32; ++d) q[d] *= scale;
      rope(q, rot + i * 32, 1.f);
      lds_store32(sv + threadIdx.x * TA_LD, q);
      if constexpr (VLDS) {
        float dd[32];
        load32(dout + vi * INNER + h * DH, dd);
        lds_store32(sb + threadIdx.x * TA_LD, dd);
      }
    }
    __syncthreads();
    if (ok) {
      const int j = i;
      float k[32], v[32], dk[32], dv[32];
      load32(qkv + vi * QKV + INNER + h * DH, k);
      rope(k, rot + j * 32, 1.f);
      load32(qkv + vi * QKV + 2 * INNER + h * DH, v);
#pragma unroll
      for (int d = 0; d < 32; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
      for (int ii = 0; ii < F; ++ii) {
        float q[32], dO[32];
        lds_load32(sv + (g * F + ii) * TA_LD, q);
        if constexpr (VLDS) {
          lds_load32(sb + (g * F + ii) * TA_LD, dO);
        } else {
          const int64_t vq = ((int64_t)b * F + ii) * HW + p;
          load32(dout + vq * INNER + h * DH, dO);
        }
        float s = 0.f, dp = 0.f;
#pragma unroll
        for (int d = 0; d < 32; ++d) { s = fmaf(q[d], k[d], s); dp = fmaf(dO[d], v[d], dp); }
        s += VLDS ? gbias[ii * F + j] : sb[ii * F + j];
        const int t2 = g * F + ii;
        const float P = expf(s - sL[t2]);
        const float dS = P * (dp - sD[t2]);
#pragma unroll
        for (int d = 0; d < 32; ++d) { dk[d] = fmaf(dS, q[d], dk[d]); dv[d] = fmaf(P, dO[d], dv[d]); }
      }
      rope(dk, rot + j * 32, -1.f);
      store32(dqkv + vi * QKV + INNER + h * DH, dk);
      store32(dqkv + vi * QKV + 2 * INNER + h * DH, dv);
    }
    __syncthreads();
  }
  // deterministic block reduction of the dbias rows over the groups
  float* outp = dbias_part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * F * F;
  for (int t = threadIdx.x; t < F * F; t += blockDim.x) {
    const int ii = t / F, j = t % F;
    float s = 0.f;
    for (int gg = 0; gg < G; ++gg) s += sacc[(gg * F + ii) * AS + j];
    outp[t] = s;
  }
}

// rel-pos bias (video_net.py:268-310): bias[h][i][j] = table[bucket(j - i)][h]
__device__ int relpos_bucket(int rel, int num_buckets, int max_distance) {
  int n = -rel;
  const int nb = num_buckets / 2;
  int ret = n < 0 ? nb : 0;
  n = n < 0 ? -n : n;
  const int max_exact = nb / 2;
  if (n < max_exact) return ret + n;
  // float32 log as in torch: (log(n/max_exact) / log(max_distance/max_exact) * (nb-max_exact)).long()
  const float lg = logf((float)n / (float)max_exact) / logf((float)max_distance / (float)max_exact) *
                   (float)(nb - max_exact);
  int large = max_exact + (int)lg;
  if (large > nb - 1) large = nb - 1;
  return ret + large;
}

__global__ void relpos_fwd_kernel(const float* __restrict__ table, float* __restrict__ bias, int F, int heads,
                                  int num_buckets, int max_distance) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= heads * F * F) return;
  const int h = t / (F * F), r = t % (F * F);
  const int i = r / F, j = r % F;
  bias[t] = table[relpos_bucket(j - i, num_buckets, max_distance) * heads + h];
}

// stage 1: dbias[h][i][j] = sum over b and the pixel-block parts (one wave per element, fixed order)
__global__ void dbias_sum_kernel(const float* __restrict__ part, float* __restrict__ dbias, int nparts_per_h, int B,
                                 int F, int heads) {
  const int t = blockIdx.x;  // element (h, i, j)
  const int h = t / (F * F), r = t % (F * F);
  float s = 0.f;
  const int n = B * nparts_per_h;
  for (int k = threadIdx.x; k < n; k += 64) {
    const int b = k / nparts_per_h, kk = k - b * nparts_per_h;
    s += part[((int64_t)(b * heads + h) * nparts_per_h + kk) * F * F + r];
  }
  s = wave_sum(s);
  if (threadIdx.x == 0) dbias[t] = s;
}

// stage 2: dtable[bucket][h] (+)= sum over (i,j) with that bucket of dbias[h][i][j]
__global__ void relpos_bwd_kernel(const float* __restrict__ dbias, float* __restrict__ dtable, int F, int heads,
                                  int num_buckets, int max_distance, int accumulate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= num_buckets * heads) return;
  const int bk = t / heads, h = t % heads;
  float s = 0.f;
  for (int i = 0; i < F; ++i)
    for (int j = 0; j < F; ++j)
      if (relpos_bucket(j - i, num_buckets, max_distance) == bk) s += dbias[(h * F + i) * F + j];
  dtable[t] = accumulate ? dtable[t] + s : s;
}

// ---------------------------------------------------------------- spatial linear attention
constexpr int SLA_TILE = 64;

// grid: x = chunk, y = frame*NH + h.  pm/pl: [frame*NH+h][chunk][32], pctx: [..][chunk][32][32]
template <typename T>
__global__ __launch_bounds__(256) void sla_ctx_partial_kernel(const T* __restrict__ qkv, float* __restrict__ pm,
                                                              float* __restrict__ pl, float* __restrict__ pctx,
                                                              int HW, int chunk) {
  __shared__ float sk[DH][SLA_TILE + 1];
  __shared__ float sv[SLA_TILE][DH + 1];
  __shared__ float smax[DH];
  const int fh = blockIdx.y;
  const int f = fh / NH, h = fh % NH;
  const int n0 = blockIdx.x * chunk, n1 = min(HW, n0 + chunk);
  const int tid = threadIdx.x;
  const int d = tid >> 3, e0 = (tid & 7) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const T* base = qkv + (int64_t)f * HW * QKV;
  for (int t0 = n0; t0 < n1; t0 += SLA_TILE) {
    // stage k[d][n], v[n][e] for the tile: 64 voxels x (32 k + 32 v); thread -> (voxel, 8-chunk)
    {
      const int vx = tid >> 2, part = tid & 3;  // 64 voxels x 4 parts of 8
      const int n = t0 + vx;
      float kk[8], vv[8];
      if (n < n1) {
        load8(base + (int64_t)n * QKV + INNER + h * DH + part * 8, kk);
        load8(base + (int64_t)n * QKV + 2 * INNER + h * DH + part * 8, vv);
      } else {
        for (int x = 0; x < 8; ++x) { kk[x] = -INFINITY; vv[x] = 0.f; }
      }
#pragma unroll
      for (int x = 0; x < 8; ++x) { sk[part * 8 + x][vx] = kk[x]; sv[vx][part * 8 + x] = vv[x]; }
    }
    __syncthreads();
    if (tid < DH) {
      float mx = -INFINITY;
      for (int x = 0; x < SLA_TILE; ++x) mx = fmaxf(mx, sk[tid][x]);
      smax[tid] = mx;
    }
    __syncthreads();
    const float mn = fmaxf(m, smax[d]);
    const float corr = (m == -INFINITY) ? 0.f : expf(m - mn);
    l *= corr;
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[x] *= corr;
    for (int x = 0; x < SLA_TILE; ++x) {
      const float pexp = expf(sk[d][x] - mn);
      l += pexp;
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[y] = fmaf(pexp, sv[x][e0 + y], acc[y]);
    }
    m = mn;
    __syncthreads();
  }
  const int64_t pi = (int64_t)fh * gridDim.x + blockIdx.x;
  if ((tid & 7) == 0) { pm[pi * DH + d] = m; pl[pi * DH + d] = l; }
#pragma unroll
  for (int y = 0; y < 4; ++y) pctx[(pi * DH + d) * DH + e0 + y] = acc[y];
}

// combine: ctx[fh][d][e] = sum_c pctx_c e^{m_c - m} / l ; ml[fh][d] = (m, l)
__global__ void sla_ctx_combine_kernel(const float* __restrict__ pm, const float* __restrict__ pl,
                                       const float* __restrict__ pctx, float* __restrict__ ctx,
                                       float* __restrict__ ml, int nchunk) {
  const int fh = blockIdx.x;
  const int d = threadIdx.x >> 5, e = threadIdx.x & 31;  // 1024 threads
  float m = -INFINITY;
  for (int c = 0; c < nchunk; ++c) m = fmaxf(m, pm[((int64_t)fh * nchunk + c) * DH + d]);
  float l = 0.f, s = 0.f;
  for (int c = 0; c < nchunk; ++c) {
    const int64_t pi = (int64_t)fh * nchunk + c;
    const float w = expf(pm[pi * DH + d] - m);
    l = fmaf(pl[pi * DH + d], w, l);
    s = fmaf(pctx[(pi * DH + d) * DH + e], w, s);
  }
  ctx[((int64_t)fh * DH + d) * DH + e] = s / l;
  if (e == 0) { ml[((int64_t)fh * DH + d) * 2] = m; ml[((int64_t)fh * DH + d) * 2 + 1] = l; }
}

// out[v][h*32+e] = sum_d ctx[f,h][d][e] * qs[d], qs = softmax_d(q) * scale
// grid: x = 64-voxel block, y = frame, z = head group of 4.  Wave w <-> head, lane <-> voxel, so
// every context read is a wave-uniform LDS broadcast.
template <typename T>
__global__ __launch_bounds__(256) void sla_out_kernel(const T* __restrict__ qkv, const float* __restrict__ ctx,
                                                      T* __restrict__ out, int HW, float scale) {
  __shared__ __attribute__((aligned(16))) float sc[4 * DH * DH];
  const int f = blockIdx.y, h0 = blockIdx.z * 4;
  const float* src = ctx + ((int64_t)f * NH + h0) * DH * DH;
  for (int e = threadIdx.x; e < 4 * DH * DH; e += 256) sc[e] = src[e];
  __syncthreads();
  const int w = threadIdx.x >> 6, h = h0 + w;
  const int p = blockIdx.x * 64 + (threadIdx.x & 63);
  if (p >= HW) return;
  const int64_t v = (int64_t)f * HW + p;
  float q[32];
  load32(qkv + v * QKV + h * DH, q);
  float mx = -INFINITY;
#pragma unroll
  for (int d = 0; d < 32; ++d) mx = fmaxf(mx, q[d]);
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < 32; ++d) { q[d] = expf(q[d] - mx); s += q[d]; }
  const float inv = scale / s;
  float o[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) o[e] = 0.f;
  const float* C = sc + w * DH * DH;
#pragma unroll 4
  for (int d = 0; d < 32; ++d) {
    const float qd = q[d] * inv;
#pragma unroll
    for (int e = 0; e < 32; e += 4) {
      const f32x4 c4 = *reinterpret_cast<const f32x4*>(C + d * DH + e);
      o[e] = fmaf(c4[0], qd, o[e]);
      o[e + 1] = fmaf(c4[1], qd, o[e + 1]);
      o[e + 2] = fmaf(c4[2], qd, o[e + 2]);
      o[e + 3] = fmaf(c4[3], qd, o[e + 3]);
    }
  }
  store32(out + v * INNER + h * DH, o);
}

// dctx partial: pd[fh][chunk][d][e] = sum_n qs[d][n] dout[e][n]
template <typename T>
__global__ __launch_bounds__(256) void sla_dctx_partial_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                               float* __restrict__ pd, int HW, int chunk,
                                                               float scale) {
  __shared__ float sq[SLA_TILE][DH + 1];
  __shared__ float sg[SLA_TILE][DH + 1];
  const int fh = blockIdx.y;
  const int f = fh / NH, h = fh % NH;
  const int n0 = blockIdx.x * chunk, n1 = min(HW, n0 + chunk);
  const int tid = threadIdx.x;
  const int d = tid >> 3, e0 = (tid & 7) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const T* qb = qkv + (int64_t)f * HW * QKV;
  const T* gb = dout + (int64_t)f * HW * INNER;
  for (int t0 = n0; t0 < n1; t0 += SLA_TILE) {
    if (tid < SLA_TILE) {
      const int n = t0 + tid;
      float q[32], gg[32];
      if (n < n1) {
        load32(qb + (int64_t)n * QKV + h * DH, q);
        load32(gb + (int64_t)n * INNER + h * DH, gg);
        float mx = -INFINITY;
        for (int x = 0; x < 32; ++x) mx = fmaxf(mx, q[x]);
        float s = 0.f;
        for (int x = 0; x < 32; ++x) { q[x] = expf(q[x] - mx); s += q[x]; }
        const float inv = scale / s;
        for (int x = 0; x < 32; ++x) q[x] *= inv;
      } else {
        for (int x = 0; x < 32; ++x) { q[x] = 0.f; gg[x] = 0.f; }
      }
      for (int x = 0; x < 32; ++x) { sq[tid][x] = q[x]; sg[tid][x] = gg[x]; }
    }
    __syncthreads();
    for (int x = 0; x < SLA_TILE; ++x) {
      const float qd = sq[x][d];
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[y] = fmaf(qd, sg[x][e0 + y], acc[y]);
    }
    __syncthreads();
  }
  const int64_t pi = (int64_t)fh * gridDim.x + blockIdx.x;
#pragma unroll
  for (int y = 0; y < 4; ++y) pd[(pi * DH + d) * DH + e0 + y] = acc[y];
}

// dctx[fh] = sum over chunks ; cvec[fh][d] = sum_e dctx[d][e]*ctx[d][e]
__global__ void sla_dctx_combine_kernel(const float* __restrict__ pd, const float* __restrict__ ctx,
                                        float* __restrict__ dctx, float* __restrict__ cvec, int nchunk) {
  const int fh = blockIdx.x;
  const int d = threadIdx.x >> 5, e = threadIdx.x & 31;
  float s = 0.f;
  for (int c = 0; c < nchunk; ++c) s += pd[(((int64_t)fh * nchunk + c) * DH + d) * DH + e];
  dctx[((int64_t)fh * DH + d) * DH + e] = s;
  float prod = s * ctx[((int64_t)fh * DH + d) * DH + e];
  // reduce over e (32 lanes of the same d share a half-wave)
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) prod += __shfl_xor(prod, o, 64);
  if (e == 0) cvec[(int64_t)fh * DH + d] = prod;
}

// per voxel, per head: dq, dk, dv.  Same wave<->head / lane<->voxel mapping as sla_out.
template <typename T>
__global__ __launch_bounds__(256) void sla_bwd_voxel_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                            const float* __restrict__ ctx,
                                                            const float* __restrict__ dctx,
                                                            const float* __restrict__ ml,
                                                            const float* __restrict__ cvec, T* __restrict__ dqkv,
                                                            int HW, float scale) {
  __shared__ __attribute__((aligned(16))) float sc[4 * DH * DH];
  __shared__ __attribute__((aligned(16))) float sdc[4 * DH * DH];
  __shared__ float sm[4 * DH], sl[4 * DH], scv[4 * DH];
  const int f = blockIdx.y, h0 = blockIdx.z * 4;
  const int64_t base = ((int64_t)f * NH + h0) * DH * DH;
  for (int e = threadIdx.x; e < 4 * DH * DH; e += 256) {
    sc[e] = ctx[base + e];
    sdc[e] = dctx[base + e];
  }
  if (threadIdx.x < 4 * DH) {
    const int64_t fhd = ((int64_t)f * NH + h0) * DH + threadIdx.x;
    sm[threadIdx.x] = ml[fhd * 2];
    sl[threadIdx.x] = ml[fhd * 2 + 1];
    scv[threadIdx.x] = cvec[fhd];
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, h = h0 + w;
  const int p = blockIdx.x * 64 + (threadIdx.x & 63);
  if (p >= HW) return;
  const int64_t v = (int64_t)f * HW + p;
  const float* C = sc + w * DH * DH;
  const float* DC = sdc + w * DH * DH;
  // ---- dq
  {
    float q[32], g[32];
    load32(qkv + v * QKV + h * DH, q);
    load32(dout + v * INNER + h * DH, g);
    float mx = -INFINITY;
#pragma unroll
    for (int d = 0; d < 32; ++d) mx = fmaxf(mx, q[d]);
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < 32; ++d) { q[d] = expf(q[d] - mx); s += q[d]; }
    const float inv = 1.f / s;
    float dsm[32], dot = 0.f;
#pragma unroll 4
    for (int d = 0; d < 32; ++d) {
      q[d] *= inv;  // sm
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < 32; e += 4) {
        const f32x4 c4 = *reinterpret_cast<const f32x4*>(C + d * DH + e);
        t = fmaf(c4[0], g[e], t);
        t = fmaf(c4[1], g[e + 1], t);
        t = fmaf(c4[2], g[e + 2], t);
        t = fmaf(c4[3], g[e + 3], t);
      }
      dsm[d] = scale * t;
      dot = fmaf(q[d], dsm[d], dot);
    }
#pragma unroll
    for (int d = 0; d < 32; ++d) dsm[d] = q[d] * (dsm[d] - dot);
    store32(dqkv + v * QKV + h * DH, dsm);
  }
  // ---- dk, dv
  {
    float k[32], vv[32];
    load32(qkv + v * QKV + INNER + h * DH, k);
    load32(qkv + v * QKV + 2 * INNER + h * DH, vv);
    float dk[32], dv[32];
#pragma unroll
    for (int e = 0; e < 32; ++e) dv[e] = 0.f;
#pragma unroll 4
    for (int d = 0; d < 32; ++d) {
      const float ks = expf(k[d] - sm[w * DH + d]) / sl[w * DH + d];
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < 32; e += 4) {
        const f32x4 c4 = *reinterpret_cast<const f32x4*>(DC + d * DH + e);
        t = fmaf(c4[0], vv[e], t);
        t = fmaf(c4[1], vv[e + 1], t);
        t = fmaf(c4[2], vv[e + 2], t);
        t = fmaf(c4[3], vv[e + 3], t);
        dv[e] = fmaf(c4[0], ks, dv[e]);
        dv[e + 1] = fmaf(c4[1], ks, dv[e + 1]);
        dv[e + 2] = fmaf(c4[2], ks, dv[e + 2]);
        dv[e + 3] = fmaf(c4[3], ks, dv[e + 3]);
      }
      dk[d] = ks * (t - scv[w * DH + d]);
    }
    store32(dqkv + v * QKV + INNER + h * DH, dk);
    store32(dqkv + v * QKV + 2 * INNER + h * DH, dv);
  }
}

template <typename F>
static int dispatch_dt(int dtype, F&& f) {
  if (dtype == CESM_DT_BF16) { f((bf16*)nullptr); return CESM_OK; }
  if (dtype == CESM_DT_F32) { f((float*)nullptr); return CESM_OK; }
  return CESM_EINVAL;
}

static int sla_chunk(int HW) {
  // ~2048 positions per chunk, multiple of the tile
  int c = 2048;
  if (HW < c) c = ((HW + SLA_TILE - 1) / SLA_TILE) * SLA_TILE;
  return c;
}

// dynamic LDS of the unfused temporal-attention kernels: RoPE table [F][32] + bias [F][F] (+ per-lane
// dbias rows [TA_T][F+1] in the backward).  F <= 32 fits the old static tables; long windows (the
// decadal F = 120 of BASELINE config 4) take one block per CU.
constexpr size_t TA_LDS_MAX = 160 * 1024;
static size_t ta_fwd_smem(int F) { return (size_t)(F * 32 + F * F) * 4; }
static size_t ta_bwd_smem(int F) { return (size_t)(F * 32 + F * F + TA_T * (F + 1)) * 4; }
template <typename K>
static void ta_allow_smem(K kernel, size_t bytes) {
  if (bytes > 48 * 1024) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

extern "C" {

int cesm_rope_table(const float* freqs, float* rot, int F, hipStream_t stream) {
  if (F < 1 || F > TA_T) return CESM_EINVAL;
  rope_table_kernel<<<(unsigned)cdiv(F * 16, 256), 256, 0, stream>>>(freqs, rot, F);
  return cesm_launch_status();
}

int cesm_relpos_fwd(const float* table, float* bias, int F, int heads, int num_buckets, int max_distance,
                    hipStream_t stream) {
  relpos_fwd_kernel<<<(unsigned)cdiv(heads * F * F, 256), 256, 0, stream>>>(table, bias, F, heads, num_buckets,
                                                                             max_distance);
  return cesm_launch_status();
}

int cesm_relpos_bwd(const float* part, int nparts_per_h, int B, float* dtable, float* ws, int F, int heads,
                    int num_buckets, int max_distance, int accumulate, hipStream_t stream) {
  dbias_sum_kernel<<<heads * F * F, 64, 0, stream>>>(part, ws, nparts_per_h, B, F, heads);
  relpos_bwd_kernel<<<(unsigned)cdiv(num_buckets * heads, 64), 64, 0, stream>>>(ws, dtable, F, heads, num_buckets,
                                                                                max_distance, accumulate);
  return cesm_launch_status();
}

// number of pixel blocks (grid.x) used by the temporal-attention kernels for HW pixels
int cesm_tattn_nblk(int F, int HW) {
  const int G = TA_T / F;
  int64_t npb = cdiv(HW, G);
  return (int)std::min<int64_t>(npb, 256);
}

int cesm_tattn_fwd(int dtype, const void* qkv, const float* bias, const float* rot, void* out, float* lse, int B,
                   int F, int HW, float scale, hipStream_t stream) {
  const bool vlds = F > 32;
  const size_t sm = vlds ? (size_t)((F * 32 + F * F + 3) & ~3) * 4 + (size_t)TA_T * TA_LD * 4 : ta_fwd_smem(F);
  if (F < 1 || F > TA_T || sm + TA_T * TA_LD * 4 > TA_LDS_MAX) return CESM_EUNSUPPORTED;
  dim3 grid(cesm_tattn_nblk(F, HW), B * NH);
  return dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    if (vlds) {
      ta_allow_smem(tattn_fwd_kernel<T, true>, sm);
      tattn_fwd_kernel<T, true><<<grid, TA_T, sm, stream>>>((const T*)qkv, bias, rot, (T*)out, lse, F, HW, scale);
    } else {
      ta_allow_smem(tattn_fwd_kernel<T>, sm);
      tattn_fwd_kernel<T><<<grid, TA_T, sm, stream>>>((const T*)qkv, bias, rot, (T*)out, lse, F, HW, scale);
    }
  }) ?: cesm_launch_status();
}

// dbias_part: B*NH*nblk*F*F floats, nblk = cesm_tattn_nblk(F, HW)
int cesm_tattn_bwd(int dtype, const void* qkv, const void* o, const void* dout, const float* lse, const float* bias,
                   const float* rot, void* dqkv, float* dbias_part, int B, int F, int HW, float scale,
                   hipStream_t stream) {
  const bool vlds = F > 32;
  const size_t sm = vlds ? (size_t)(F * 32 + TA_T * TA_LD + TA_T * (F + 1)) * 4 : ta_bwd_smem(F);
  if (F < 1 || F > TA_T || sm + (TA_T * TA_LD + 2 * TA_T) * 4 > TA_LDS_MAX) return CESM_EUNSUPPORTED;
  dim3 grid(cesm_tattn_nblk(F, HW), B * NH);
  return dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    if (vlds) {
      ta_allow_smem(tattn_bwd_kernel<T, true>, sm);
      tattn_bwd_kernel<T, true><<<grid, TA_T, sm, stream>>>((const T*)qkv, (const T*)o, (const T*)dout, lse, bias, rot,
                                                            (T*)dqkv, dbias_part, F, HW, scale);
    } else {
      ta_allow_smem(tattn_bwd_kernel<T>, sm);
      tattn_bwd_kernel<T><<<grid, TA_T, sm, stream>>>((const T*)qkv, (const T*)o, (const T*)dout, lse, bias, rot,
                                                     (T*)dqkv, dbias_part, F, HW, scale);
    }
  }) ?: cesm_launch_status();
}

int cesm_sla_nchunk(int HW) { return (int)cdiv(HW, sla_chunk(HW)); }

// Nf = number of frames (B*F); ws: floats >= Nf*NH*nchunk*(32+32+1024); ctx [Nf][NH][32][32], ml [Nf][NH][32][2]
int cesm_sla_fwd(int dtype, const void* qkv, void* out, float* ctx, float* ml, float* ws, int Nf, int HW, float scale,
                 hipStream_t stream) {
  const int chunk = sla_chunk(HW);
  const int nchunk = (int)cdiv(HW, chunk);
  float* pm = ws;
  float* pl = pm + (int64_t)Nf * NH * nchunk * DH;
  float* pctx = pl + (int64_t)Nf * NH * nchunk * DH;
  return dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    sla_ctx_partial_kernel<T><<<dim3(nchunk, Nf * NH), 256, 0, stream>>>((const T*)qkv, pm, pl, pctx, HW, chunk);
    sla_ctx_combine_kernel<<<Nf * NH, 1024, 0, stream>>>(pm, pl, pctx, ctx, ml, nchunk);
    sla_out_kernel<T><<<dim3((unsigned)cdiv(HW, 64), Nf, 2), 256, 0, stream>>>((const T*)qkv, ctx, (T*)out, HW,
                                                                                scale);
  }) ?: cesm_launch_status();
}

// ws: floats >= Nf*NH*nchunk*1024 + Nf*NH*(1024+32)
int cesm_sla_bwd(int dtype, const void* qkv, const void* dout, const float* ctx, const float* ml, void* dqkv,
                 float* ws, int Nf, int HW, float scale, hipStream_t stream) {
  const int chunk = sla_chunk(HW);
  const int nchunk = (int)cdiv(HW, chunk);
  float* pd = ws;
  float* dctx = pd + (int64_t)Nf * NH * nchunk * DH * DH;
  float* cvec = dctx + (int64_t)Nf * NH * DH * DH;
  return dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    sla_dctx_partial_kernel<T><<<dim3(nchunk, Nf * NH), 256, 0, stream>>>((const T*)qkv, (const T*)dout, pd, HW,
                                                                           chunk, scale);
    sla_dctx_combine_kernel<<<Nf * NH, 1024, 0, stream>>>(pd, ctx, dctx, cvec, nchunk);
    sla_bwd_voxel_kernel<T><<<dim3((unsigned)cdiv(HW, 64), Nf, 2), 256, 0, stream>>>(
        (const T*)qkv, (const T*)dout, ctx, dctx, ml, cvec, (T*)dqkv, HW, scale);
  }) ?: cesm_launch_status();
}

}  // extern "C"
