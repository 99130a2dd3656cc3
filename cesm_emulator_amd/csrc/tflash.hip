// Temporal attention core on MFMA for the unfused path (bf16): long windows (F = 120, BASELINE config 4) and
// the C >= 256 levels.  Same contract as tattn_fwd / tattn_bwd in attn.hip (video_net.py:403-454):
//   per (sample b, pixel p, head h): q' = scale R_f q_f, k' = R_f k_f (RoPE, rotary_embedding.py:35-48),
//   S[i][j] = q'_i . k'_j + bias[h][i][j], P = softmax_j S, O_i = sum_j P_ij v_j.
// One wave owns one (pixel, head): F <= 128 frames = NT 16-frame tiles, every q.k product a 16x16x32 MFMA
// (K = the 32 head dims).  The transposed orientation is used throughout: S^T tiles put a query column in
// each lane group, so the softmax over keys is an in-lane loop + a 4-lane-group reduction, and two key
// tiles of P^T in MFMA D layout are directly a B operand through the k-slot map (slot (g, j < 4) <-> key
// 4g + j, (g, 4 + j) <-> 16 + 4g + j); the matching A operands (V^T, K'^T, Q'^T, dO^T) are gathered from
// LDS-staged rows with the hardware transpose read.
// The rel-pos bias depends on j - i only: it is read from a per-head table by offset (2F - 1 entries), and
// its gradient is accumulated by offset in registers (the offset of every element a lane holds is fixed by
// the lane, the register index and the (query tile, key tile) pair) and reduced to buckets afterwards.
// Backward = two kernels: dq (query tiles outer; D_i = dO_i . O_i; dbias) and dk / dv (key tiles outer).
// Every kernel here is capped at 256 registers (>= 2 waves per SIMD): with a 512-register budget the compiler
// selects the AGPR form of the MFMAs, and the score tiles -- consumed by VALU right away -- then cost 4
// v_accvgpr_read each and share one accumulator quad, serialising the MFMAs behind s_nop waits.
#include "common.h"
#include "cesm_hip.h"

namespace {

constexpr int NH = 8, DH = 32, INNER = 256, QKV = 768;
constexpr float LOG2E = 1.4426950408889634f;
constexpr int TF_LD = 40;     // staged-row stride (bf16): 80-B rows
constexpr int TF_MAXT = 8;    // 16-frame tiles: F <= 128
// row stride (floats) of the LDS table of frames 0 .. 15's RoPE rows: lane (g, lr) reads row lr at float 8g (+4) or
// (8t + 2g) * 2 -- with 32-float rows 16 lanes of a ds_read_b128 group hit 4 bank sets (16 cycles, 4x); with 40,
// 8 and 4 cycles (tools/lds_banks.py)
constexpr int TF_RBS = 40;

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
__device__ __forceinline__ bf16x8 pack_kslot(const float* t0, const float* t1) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (bf16)t0[j];
    r[4 + j] = (bf16)t1[j];
  }
  return r;
}
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// RoPE (cos, sin) of the 4 dim pairs 4g..4g+3 of frame f
__device__ __forceinline__ void rot8_load(const float* __restrict__ rot, int f, int g, float* cs) {
  const f32x4 c0 = *reinterpret_cast<const f32x4*>(rot + (f * 16 + 4 * g) * 2);
  const f32x4 c1 = *reinterpret_cast<const f32x4*>(rot + (f * 16 + 4 * g + 2) * 2);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    cs[i] = c0[i];
    cs[4 + i] = c1[i];
  }
}
// the 8 dims of a raw row chunk rotated with rot8_load's coefficients, times `scale`
__device__ __forceinline__ bf16x8 rope8(const bf16x8 v, const float* cs, float scale) {
  bf16x8 o;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float c = cs[2 * u], s = cs[2 * u + 1];
    const float a = (float)v[2 * u], b = (float)v[2 * u + 1];
    o[2 * u] = (bf16)((a * c - b * s) * scale);
    o[2 * u + 1] = (bf16)((b * c + a * s) * scale);
  }
  return o;
}

// Buffer-resource addressing of a 16-frame tile: the tile's base is wave-uniform (SGPRs), a lane's
// frame row is a 32-bit byte offset lr * HW * rowbytes (< 2^31: checked on the host), and the resource ends
// after the tile's last valid frame, so loads of frames >= F return zeros and stores to them are dropped --
// no 64-bit lane address math and no predicate branch per tile (the 64-bit math was ~60 of the forward's
// ~320 VALU per query tile).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// `nvalid` counts the valid frames from the tile's first one; the resource covers at most `maxrows` of them (16 for a
// query / output tile: a 120-frame window at 192x288 would otherwise span 119 * HW * 1536 B, past the 32-bit
// num_records, which then wrapped and dropped rows of the tile).  The host bounds maxrows * fstride_b < 2^31.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* base, int nvalid, int64_t fstride_b, int rowb,
                                                            int maxrows = 16) {
  nvalid = nvalid < maxrows ? nvalid : maxrows;
  const int64_t n = nvalid > 0 ? (int64_t)(nvalid - 1) * fstride_b + rowb : 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ bf16x8 buf_ld16(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void buf_rot8(__amdgpu_buffer_rsrc_t r, int off, float* cs) {
  const f32x4 c0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  const f32x4 c1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    cs[i] = c0[i];
    cs[4 + i] = c1[i];
  }
}
__device__ __forceinline__ void buf_st4b(__amdgpu_buffer_rsrc_t r, int off, const float* v) {
  bf16x4 a = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, a), r, off, 0, 0);
}

// 8 head dims 8g..8g+7 of one frame row (16-B load), RoPE-rotated by frame f when rot != null, times `scale`
__device__ __forceinline__ bf16x8 row_frag(const bf16* p, const float* __restrict__ rot, int f, int g, float scale,
                                           bool ok) {
  const bf16x8 v = ld16(p);
  bf16x8 o = zero8();
  if (rot) {
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(rot + (f * 16 + 4 * g) * 2);      // pairs 4g, 4g+1
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(rot + (f * 16 + 4 * g + 2) * 2);  // pairs 4g+2, 4g+3
    const float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float c = cs[2 * u], s = cs[2 * u + 1];
      const float a = (float)v[2 * u], b = (float)v[2 * u + 1];
      o[2 * u] = (bf16)(ok ? (a * c - b * s) * scale : 0.f);
      o[2 * u + 1] = (bf16)(ok ? (b * c + a * s) * scale : 0.f);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = ok ? v[e] : (bf16)0.f;
  }
  return o;
}

// A operand with rows = 16 head dims (c0 .. c0+15) and k-slots = the 32 frames of pair s of a staged
// [frames][TF_LD] tile: lane (g, i) <- tile[32s + kslot(g, j)][c0 + i]
__device__ __forceinline__ bf16x8 tr_pair(const bf16* tile, int s, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + (32 * s + 4 * g + q) * TF_LD + c0 + 4 * p));
  const s16x4 b =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tile + (32 * s + 16 + 4 * g + q) * TF_LD + c0 + 4 * p));
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = __builtin_bit_cast(bf16, (short)a[j]);
    r[4 + j] = __builtin_bit_cast(bf16, (short)b[j]);
  }
  return r;
}

// R^T (inverse rotation) of dims d0 .. d0+3 (two pairs) of frame f, times `scale`
__device__ __forceinline__ void rope4_inv(float* v, const float* __restrict__ rot, int f, int d0, float scale) {
  const f32x4 cs = *reinterpret_cast<const f32x4*>(rot + (f * 16 + d0 / 2) * 2);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const float c = cs[2 * u], s = cs[2 * u + 1];
    const float a = v[2 * u], b = v[2 * u + 1];
    v[2 * u] = (a * c + b * s) * scale;
    v[2 * u + 1] = (b * c - a * s) * scale;
  }
}

__device__ __forceinline__ void store4b(bf16* p, const float* v) {
  bf16x4 a = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  *reinterpret_cast<bf16x4*>(p) = a;
}

// Score-tile bias table: tab[c][k] = bias(n) for n = sign * (k + c - 16 NT) (log2 units, 0 for |n| >= F), four
// copies shifted by c = 0..3.  An MFMA D fragment's four consecutive offsets (register r of lane (g, lr) in the
// (row tile a, column tile b) block: n = 16 (b - a) + 4g - lr + r) are then ONE aligned 16-B read at
// btab_lane(..) + 16 (b - a): lane-constant base, immediate offset per tile pair -- instead of an index
// computation, clamp and 4-B read per element.  Every offset a padded row / column can form is in range.
template <int NT>
__device__ __forceinline__ void load_btab(const float* __restrict__ bias, float* tab, int h, int F, int sign, int tid,
                                          int nthr) {
  constexpr int TL = 32 * NT;
  for (int e = tid; e < 4 * TL; e += nthr) {
    const int c = e / TL, k = e - c * TL;
    const int n = sign * (k + c - 16 * NT);
    float v = 0.f;
    if (n > -F && n < F) {
      const int i = n < 0 ? -n : 0, j = i + n;
      v = bias[((int64_t)h * F + i) * F + j] * LOG2E;
    }
    tab[e] = v;
  }
}
template <int NT>
__device__ __forceinline__ const float* btab_lane(const float* tab, int lr, int g) {
  const int e0 = 4 * g - lr + 16 * NT, c = e0 & 3;  // e0 - c >= 0 and e0 + 16 (NT - 1) + 3 < 32 NT
  return tab + c * 32 * NT + (e0 - c);
}
// Block -> (4-pixel group, head) of the per-pixel kernels (fwd, bwd_kv): grid (8 * 8 * cdiv(groups, 8), B).
// A head's q / k / v are 64 B of the voxel's 1536-B qkv row, half a 128-B line.  Workgroups are dealt to the
// 8 XCDs round-robin (linear id mod 8), so the 8 blocks an XCD receives back to back (ids L, L + 8, ...) are
// the 8 heads of one pixel group: every line is fetched once into that XCD's L2 and used whole.  (One head per
// grid row instead fetched each line twice from HBM: the head-pair partner ran 1/8 of the grid later.)
// (Round 3, head-major grid instead: forward +18 %.)
__device__ __forceinline__ void tf_block(int& grp, int& h) {
  const int L = blockIdx.x, j = L >> 3;
  h = j & 7;
  grp = (j >> 3) * 8 + (L & 7);
}
constexpr int TF_VH = 2;  // forward V staging: key-tile pairs per part (4 = all at F = 128)
static unsigned tf_grid_x(int HW) { return (unsigned)(64 * cdiv(cdiv(HW, 4), 8)); }

// padded query rows: their lse makes every P entry exactly 0 (exp2(x - 1e30) = 0 for any finite x)
constexpr float TF_LSE_PAD = 1e30f;

// ------------------------------------------------------------------------------------------------ forward
// grid (tf_grid_x(HW), B), 256 threads: wave = one pixel of one (sample, head) (tf_block); waves_per_eu(2): a
// 256-register budget, VGPR-form MFMAs.

// Round 5 form of the forward: every global load of the wave is issued up front -- the raw K and Q
// rows of all tiles through tile resources (frames >= F read as zeros) and the V rows of the first staging part --
// and the RoPE coefficients come by angle addition (frame 16 a + lr = the block's row of frame 16 a composed with the
// row of frame lr, two small LDS tables; the fused backward uses the same coefficients).  No load is issued after the
// wave's first O store: vmcnt counts loads and stores in order, and in the round 2-4 form (removed in round 6) every
// query tile's q and RoPE loads waited behind the previous tile's stores, and the K' prologue waited once per key tile
// (192 x 288, F = 120: 4.63 -> 4.12 ms).
template <int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void tflash_fwd2_kernel(
    const bf16* __restrict__ qkv, const float* __restrict__ bias, const float* __restrict__ rot, bf16* __restrict__ out,
    float* __restrict__ lse, int F, int HW, float scale, int pm) {
  constexpr int NP = (NT + 1) / 2;
  constexpr int VH = NP < TF_VH ? NP : TF_VH, NVR = 32 * VH;
  __shared__ __attribute__((aligned(16))) float btab[4 * 32 * NT];
  __shared__ __attribute__((aligned(16))) float rtab[32 * NT];    // RoPE (cos, sin) rows of frames 16 a
  __shared__ __attribute__((aligned(16))) float rbase[16 * TF_RBS];  // ... of frames 0 .. 15 (0 past F)
  __shared__ __attribute__((aligned(16))) bf16 vst[4][NVR * TF_LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, lr = lane & 15, g = lane >> 4;
  int grp, h;
  tf_block(grp, h);
  const int b = blockIdx.y;
  if (grp * 4 >= HW) return;  // whole block (padded groups)
  load_btab<NT>(bias, btab, h, F, 1, tid, 256);
  for (int e = tid; e < 32 * NT; e += 256) rtab[e] = rot[(e >> 5) * 16 * 32 + (e & 31)];
  for (int e = tid; e < 16 * 32; e += 256) rbase[(e >> 5) * TF_RBS + (e & 31)] = e < F * 32 ? rot[e] : 0.f;
  __syncthreads();
  const int p = grp * 4 + __builtin_amdgcn_readfirstlane(wid);  // wave-uniform (buffer bases in SGPRs)
  if (p >= HW) return;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  const int64_t row0 = (int64_t)b * F * HW + p;
  const int64_t qrow0 = pm ? ((int64_t)b * HW + p) * F : row0;
  const int qfs = pm ? 1 : HW;
  const int fs_qkv = qfs * QKV * 2;  // 16 rows < 2^31 B: checked on the host
  const int lo = lr * fs_qkv + (h * DH + g * 8) * 2;
  bf16x8 kr[NT], qr[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(qkv + (qrow0 + (int64_t)t * 16 * qfs) * QKV, F - t * 16, (int64_t)fs_qkv,
                                               QKV * 2);
    kr[t] = buf_ld16(rs, lo + INNER * 2);
    qr[t] = buf_ld16(rs, lo);
  }
  bf16* vs = vst[wid];
  auto vload = [&](int s0, bf16x8* vraw) {
#pragma unroll
    for (int i = 0; i < NVR * 4 / 64; ++i) {
      const int e = lane + 64 * i, fl = e >> 2, c = e & 3, f = 32 * s0 + fl;
      vraw[i] = ld16(qkv + (qrow0 + (int64_t)(f < F ? f : 0) * qfs) * QKV + 2 * INNER + h * DH + c * 8);
      if (f >= F) vraw[i] = zero8();
    }
  };
  bf16x8 vraw[NVR * 4 / 64];
  vload(0, vraw);
  const float* rb = rbase + lr * TF_RBS + 8 * g;
  auto cs8 = [&](int a, float* cs) {  // pairs 4g .. 4g + 3 of frame 16 a + lr
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float cb = rb[2 * u], sb = rb[2 * u + 1], ct = rtab[a * 32 + 8 * g + 2 * u], st = rtab[a * 32 + 8 * g + 2 * u + 1];
      cs[2 * u] = cb * ct - sb * st;
      cs[2 * u + 1] = sb * ct + cb * st;
    }
  };
  bf16x8 kf[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    float cs[8];
    cs8(kt, cs);
    kf[kt] = rope8(kr[kt], cs, 1.f);
  }
  bf16x8 vf[NP][2];
#pragma unroll
  for (int s0 = 0; s0 < NP; s0 += VH) {
    if (s0) {
      wsync();  // previous part's transposed reads done
      vload(s0, vraw);
    }
#pragma unroll
    for (int i = 0; i < NVR * 4 / 64; ++i) {
      const int e = lane + 64 * i, fl = e >> 2, c = e & 3;
      *reinterpret_cast<bf16x8*>(vs + fl * TF_LD + c * 8) = vraw[i];
    }
    wsync();
#pragma unroll
    for (int s = s0; s < s0 + VH && s < NP; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) vf[s][t] = tr_pair(vs, s - s0, t * 16, lane);
  }
  const float* bl = btab_lane<NT>(btab, lr, g);
  float kmask[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) kmask[r] = 16 * (NT - 1) + 4 * g + r < F ? 0.f : -INFINITY;
  const int o_off = (lr * HW * INNER + 4 * g) * 2;
#pragma unroll
  for (int qt = 0; qt < NT; ++qt) {
    const int nq = F - qt * 16;
    float cs[8];
    cs8(qt, cs);
    const bf16x8 qf = rope8(qr[qt], cs, scale);  // frames >= F: zeros
    const float* bq = bl - 16 * qt;
    float sc[2 * NP][4];
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2 * NP; ++kt) {
      if (kt < NT) {
        const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt < NT ? kt : 0], qf, z4, 0, 0, 0);
        const f32x4 bo = *reinterpret_cast<const f32x4*>(bq + 16 * kt);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sc[kt][r] = fmaf(st[r], LOG2E, bo[r]);
          if (kt == NT - 1) sc[kt][r] += kmask[r];
          m = fmaxf(m, sc[kt][r]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[kt][r] = -INFINITY;
      }
    }
    const float mm = grp4_max(m);  // finite: key 0 is valid for every query row
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2 * NP; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sc[kt][r] = __builtin_amdgcn_exp2f(sc[kt][r] - mm);  // exp2(-inf) = 0
        l += sc[kt][r];
      }
    l = grp4_sum(l);
    f32x4 ot[2] = {z4, z4};
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      const bf16x8 pb = pack_kslot(sc[2 * s], sc[2 * s + 1]);
#pragma unroll
      for (int t = 0; t < 2; ++t) ot[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[s][t], pb, ot[t], 0, 0, 0);
    }
    // stores of frames >= F fall outside the resources and are dropped
    const float inv = __builtin_amdgcn_rcpf(l);
    const __amdgpu_buffer_rsrc_t ors =
        tile_rsrc(out + (row0 + (int64_t)qt * 16 * HW) * INNER + h * DH, nq, (int64_t)HW * INNER * 2, DH * 2);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float o4[4] = {ot[t][0] * inv, ot[t][1] * inv, ot[t][2] * inv, ot[t][3] * inv};
      buf_st4b(ors, o_off + t * 32, o4);
    }
    if (lse) {
      const __amdgpu_buffer_rsrc_t lrs = tile_rsrc(lse + (((int64_t)b * NH + h) * HW + p) * F + qt * 16, nq, 4, 4);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, mm + log2f(l)), lrs,
                                            g == 0 ? lr * 4 : 0x7ffffff0, 0, 0);
    }
  }
}

// ------------------------------------------------------------------------------------------------ backward, dq
// grid (nblk, B * 8), 64*NT threads: wave w = query tile w of the block's current pixel (grid-stride over pixels),
// the pixel's K' and V rows staged once in LDS for all waves.  Writes dq into dqkv, D_i = dO_i . O_i into dbuf
// [B][8][HW][F], and per-block dbias-by-offset partials part[(b*8 + h)][blk][2F - 1].  With the query tile
// fixed per wave, the dbias accumulator of (r, kt) holds one diagonal kt - qt for every pixel: static registers.
// Round 6: only the F < 8 windows take this two-kernel backward (the one-pass fused kernel takes every longer one);
// D_i = sum_j P_ij dP_ij keeps the F = 1 rel-pos bias gradient exactly 0.  (The single-pass variant with D = dO . O
// from the forward's output, round 3's TF_DO for small F > 16 levels, went with the fused kernel.)
template <int NT>
__global__ __launch_bounds__(64 * NT) __attribute__((amdgpu_waves_per_eu(2))) void tflash_bwd_q_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ bias, const float* __restrict__ rot,
    bf16* __restrict__ dqkv, float* __restrict__ dbuf, float* __restrict__ part, int F, int HW, float scale, int pm) {
  constexpr int NP = (NT + 1) / 2, NR = 32 * NP, NTH = 64 * NT;
  __shared__ __attribute__((aligned(16))) float btab[4 * 32 * NT];
  __shared__ float dacc[2 * 16 * TF_MAXT];
  __shared__ __attribute__((aligned(16))) bf16 ks[NR * TF_LD];
  __shared__ __attribute__((aligned(16))) bf16 vs[NR * TF_LD];
  const int tid = threadIdx.x, lane = tid & 63, qt = tid >> 6, lr = lane & 15, g = lane >> 4;
  const int b = blockIdx.y >> 3, h = blockIdx.y & 7;
  load_btab<NT>(bias, btab, h, F, 1, tid, NTH);
  for (int e = tid; e < 2 * 16 * TF_MAXT; e += NTH) dacc[e] = 0.f;
  for (int e = tid; e < (NR - 16 * NT) * 4; e += NTH) {  // rows past the last key tile stay zero
    const int f = 16 * NT + (e >> 2), c = e & 3;
    *reinterpret_cast<bf16x8*>(ks + f * TF_LD + c * 8) = zero8();
  }
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  float dba[4][NT];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) dba[r][kt] = 0.f;
  const int fq = qt * 16 + lr;
  const bool okq = fq < F;
  const float* bq = btab_lane<NT>(btab, lr, g) - 16 * qt;
  bool kok[4];  // keys of the last key tile below F
#pragma unroll
  for (int r = 0; r < 4; ++r) kok[r] = 16 * (NT - 1) + 4 * g + r < F;

  // Software pipeline over the block's pixels: the next pixel's raw rows are loaded into registers while the
  // current one is computed (one block per CU at 2 waves per SIMD: a load issued at the top of an iteration
  // was fully exposed).  Each thread stages exactly one 16-B chunk of K' and of V per pixel (16 NT frames x 4
  // chunks = NTH); its frame, and so its RoPE coefficients, are the same for every pixel, as are the query's.
  const int sf = tid >> 2, sc = tid & 3;
  const bool sok = sf < F;
  const int sfc = sok ? sf : 0, fqc = okq ? fq : 0;
  float kcs[8], qcs[8];
  rot8_load(rot, sfc, sc, kcs);
  rot8_load(rot, fqc, g, qcs);
  bf16x8 kraw = zero8(), vraw = zero8(), qraw = zero8(), draw = zero8();
  float lraw = 0.f;
  // qkv / dqkv rows frame-major or pixel-major (pm); dout / o frame-major
  const int qfs = pm ? 1 : HW;
  auto qrow = [&](int pp) { return pm ? ((int64_t)b * HW + pp) * F : (int64_t)b * F * HW + pp; };
  auto fetch = [&](int pp) {
    const int64_t r0 = (int64_t)b * F * HW + pp, q0 = qrow(pp);
    const int64_t rs = (q0 + (int64_t)sfc * qfs) * QKV + h * DH + sc * 8;
    kraw = ld16(qkv + rs + INNER);
    vraw = ld16(qkv + rs + 2 * INNER);
    const int64_t vq = r0 + (int64_t)fqc * HW;
    qraw = ld16(qkv + (q0 + (int64_t)fqc * qfs) * QKV + h * DH + g * 8);
    draw = ld16(dout + vq * INNER + h * DH + g * 8);
    lraw = lse[(((int64_t)b * NH + h) * HW + pp) * F + fqc];
  };
  if ((int)blockIdx.x < HW) fetch(blockIdx.x);

  for (int p = blockIdx.x; p < HW; p += gridDim.x) {
    const int64_t row0 = (int64_t)b * F * HW + p, qrow0 = qrow(p);
    __syncthreads();  // previous pixel's rows consumed
    bf16x8 qf, dof;
    float Li;
    {
      *reinterpret_cast<bf16x8*>(ks + sf * TF_LD + sc * 8) = sok ? rope8(kraw, kcs, 1.f) : zero8();
      *reinterpret_cast<bf16x8*>(vs + sf * TF_LD + sc * 8) = sok ? vraw : zero8();
      // padded query rows: finite clamped data, P = 0 through Li (so D = dS = 0 there)
      qf = rope8(qraw, qcs, scale);
      dof = draw;
      Li = okq ? lraw : TF_LSE_PAD;
    }
    if (p + (int)gridDim.x < HW) fetch(p + gridDim.x);
    __syncthreads();  // rows staged
    // pass 1: P^T and dP^T of every key tile, D_i = sum_j P_ij dP_ij (exact: at F = 1 the bias gradient is 0)
    float pt[NT][4], dpt[NT][4];
    float D = 0.f;
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      const bf16x8 kf = ld16(ks + (kt * 16 + lr) * TF_LD + g * 8);
      const bf16x8 vf = ld16(vs + (kt * 16 + lr) * TF_LD + g * 8);
      const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, z4, 0, 0, 0);   // S'^T
      const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, dof, z4, 0, 0, 0);  // dP^T
      const f32x4 bo = *reinterpret_cast<const f32x4*>(bq + 16 * kt);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pt[kt][r] = __builtin_amdgcn_exp2f(fmaf(st[r], LOG2E, bo[r]) - Li);
        if (kt == NT - 1) pt[kt][r] = kok[r] ? pt[kt][r] : 0.f;
        dpt[kt][r] = dp[r];
        D = fmaf(pt[kt][r], dp[r], D);
      }
    }
    D = grp4_sum(D);
    if (okq && g == 0) dbuf[(((int64_t)b * NH + h) * HW + p) * F + fq] = D;
    // pass 2: dS^T = P^T (dP^T - D) -> dbias, dQ'^T = K'^T dS^T
    f32x4 dqt[2] = {z4, z4};
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      float dsv[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int kt = 2 * s + u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ds = kt < NT ? pt[kt < NT ? kt : 0][r] * (dpt[kt < NT ? kt : 0][r] - D) : 0.f;
          dsv[u][r] = ds;
          if (kt < NT) dba[r][kt < NT ? kt : 0] += ds;
        }
      }
      const bf16x8 db = pack_kslot(dsv[0], dsv[1]);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        dqt[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_pair(ks, s, t * 16, lane), db, dqt[t], 0, 0, 0);
    }
    if (okq) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int d0 = t * 16 + 4 * g;
        float v4[4] = {dqt[t][0], dqt[t][1], dqt[t][2], dqt[t][3]};
        rope4_inv(v4, rot, fq, d0, scale);  // dq = scale R^T dQ'
        store4b(dqkv + (qrow0 + (int64_t)fq * qfs) * QKV + h * DH + d0, v4);
      }
    }
  }
  // dbias partials by offset n = 16 (kt - qt) + 4g + r - lr: the lanes' accumulators are staged one key tile at a
  // time and each offset sums its contributions in a fixed (kt, qt, g, r) order, so the block's row is the same on
  // every run (LDS float atomics over lanes and waves were not)
  __shared__ float dstage[TF_MAXT][4][64];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) dstage[qt][r][lane] = dba[r][kt];
    __syncthreads();
    for (int e = tid; e < 2 * F - 1; e += NTH) {
      const int n = e - (F - 1);
      float a = dacc[e];
      for (int q = 0; q < NT; ++q)
        for (int gg = 0; gg < 4; ++gg)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int l = 16 * (kt - q) + 4 * gg + r - n;
            if (l >= 0 && l < 16) a += dstage[q][r][gg * 16 + l];
          }
      dacc[e] = a;
    }
  }
  __syncthreads();
  for (int e = tid; e < 2 * F - 1; e += NTH)
    part[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (2 * F - 1) + e] = dacc[e];
}

// ------------------------------------------------------------------------------------------------ backward, dk dv
// grid (tf_grid_x(HW), B), 256 threads: wave = one pixel (tf_block); key tiles outer, query-tile pairs inner
template <int NT>
__global__ __launch_bounds__(256, 2) void tflash_bwd_kv_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ dbuf, const float* __restrict__ bias, const float* __restrict__ rot,
    bf16* __restrict__ dqkv, int F, int HW, float scale, int pm) {
  constexpr int NP = (NT + 1) / 2, NR = 32 * NP;
  __shared__ __attribute__((aligned(16))) float btab[4 * 32 * NT];
  __shared__ __attribute__((aligned(16))) bf16 stg[4][NR * TF_LD];
  __shared__ __attribute__((aligned(16))) float lds_l[4][NR], lds_d[4][NR];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, lr = lane & 15, g = lane >> 4;
  int grp, h;
  tf_block(grp, h);
  const int b = blockIdx.y;
  if (grp * 4 >= HW) return;  // whole block (padded groups)
  load_btab<NT>(bias, btab, h, F, -1, tid, 256);  // rows = queries here: offsets key - query = -(q - key)
  __syncthreads();
  const int p = grp * 4 + wid;
  if (p >= HW) return;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  const int64_t row0 = (int64_t)b * F * HW + p;
  const int64_t qrow0 = pm ? ((int64_t)b * HW + p) * F : row0;  // qkv / dqkv rows (pm: pixel-major)
  const int qfs = pm ? 1 : HW;
  bf16* st = stg[wid];
  float* Ls = lds_l[wid];
  float* Ds = lds_d[wid];
  for (int e = lane; e < NR; e += 64) {
    const bool ok = e < F;
    const int64_t si = (((int64_t)b * NH + h) * HW + p) * F + (ok ? e : 0);
    Ls[e] = ok ? lse[si] : TF_LSE_PAD;  // padded query rows: P = dS = 0, no mask in the loop
    Ds[e] = ok ? dbuf[si] : 0.f;
  }
  for (int e = lane; e < (NR - 16 * NT) * 4; e += 64) {
    const int f = 16 * NT + (e >> 2), c = e & 3;
    *reinterpret_cast<bf16x8*>(st + f * TF_LD + c * 8) = zero8();
  }
  // query-row operands: Q' (rotated, scaled) and dO as A fragments, and their k-slot transposes
  bf16x8 qa[NT], da[NT], qtf[NP][2], dtf[NP][2];
#pragma unroll
  for (int qt = 0; qt < NT; ++qt) {
    const int f = qt * 16 + lr;
    const bool ok = f < F;
    const int64_t vq = row0 + (int64_t)(ok ? f : 0) * HW;
    qa[qt] = row_frag(qkv + (qrow0 + (int64_t)(ok ? f : 0) * qfs) * QKV + h * DH + g * 8, rot, ok ? f : 0, g, scale,
                      true);  // padded: P = dS = 0
    da[qt] = row_frag(dout + vq * INNER + h * DH + g * 8, nullptr, 0, g, 1.f, true);
    *reinterpret_cast<bf16x8*>(st + f * TF_LD + g * 8) = qa[qt];
  }
  wsync();
#pragma unroll
  for (int s = 0; s < NP; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t) qtf[s][t] = tr_pair(st, s, t * 16, lane);
  wsync();
#pragma unroll
  for (int qt = 0; qt < NT; ++qt) *reinterpret_cast<bf16x8*>(st + (qt * 16 + lr) * TF_LD + g * 8) = da[qt];
  wsync();
#pragma unroll
  for (int s = 0; s < NP; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t) dtf[s][t] = tr_pair(st, s, t * 16, lane);

  const float* bl = btab_lane<NT>(btab, lr, g);
  // key tile kt + 1's raw K / V rows and RoPE coefficients are loaded while tile kt is computed
  bf16x8 kraw, vraw;
  float kcs[8];
  auto fetch = [&](int t) {
    const int fk = t * 16 + lr, fkc = fk < F ? fk : 0;
    const int64_t rk = (qrow0 + (int64_t)fkc * qfs) * QKV + h * DH + g * 8;
    kraw = ld16(qkv + rk + INNER);
    vraw = ld16(qkv + rk + 2 * INNER);
    rot8_load(rot, fkc, g, kcs);
  };
  fetch(0);
  for (int kt = 0; kt < NT; ++kt) {
    const int fk = kt * 16 + lr;
    const bool okk = fk < F;  // padded key columns: finite garbage, not stored
    const float* bk = bl - 16 * kt;
    const bf16x8 kb = rope8(kraw, kcs, 1.f);  // K'^T col
    const bf16x8 vb = vraw;                   // V^T col
    if (kt + 1 < NT) fetch(kt + 1);
    f32x4 dk[2] = {z4, z4}, dv[2] = {z4, z4};
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      float pv[2][4], dsv[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * s + u;
        if (qt < NT) {
          const f32x4 sq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[qt], kb, z4, 0, 0, 0);  // S'[q][key]
          const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[qt], vb, z4, 0, 0, 0);  // dP[q][key]
          const f32x4 bo = *reinterpret_cast<const f32x4*>(bk + 16 * qt);
          const f32x4 lq = *reinterpret_cast<const f32x4*>(Ls + qt * 16 + 4 * g);
          const f32x4 dq = *reinterpret_cast<const f32x4*>(Ds + qt * 16 + 4 * g);
          // two elements per VALU op (v_pk_fma / v_pk_add / v_pk_mul_f32), same operations and order as below
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const f32x2 s2 = {sq[r], sq[r + 1]}, b2 = {bo[r], bo[r + 1]}, l2 = {lq[r], lq[r + 1]};
            const f32x2 x2 = __builtin_elementwise_fma(s2, f32x2{LOG2E, LOG2E}, b2) - l2;
            const f32x2 p2 = {__builtin_amdgcn_exp2f(x2[0]), __builtin_amdgcn_exp2f(x2[1])};
            const f32x2 d2 = p2 * (f32x2{dp[r], dp[r + 1]} - f32x2{dq[r], dq[r + 1]});
            pv[u][r] = p2[0];
            pv[u][r + 1] = p2[1];
            dsv[u][r] = d2[0];
            dsv[u][r + 1] = d2[1];
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) pv[u][r] = dsv[u][r] = 0.f;
        }
      }
      const bf16x8 pb = pack_kslot(pv[0], pv[1]);
      const bf16x8 db = pack_kslot(dsv[0], dsv[1]);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        dv[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dtf[s][t], pb, dv[t], 0, 0, 0);  // dV^T[d][key]
        dk[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qtf[s][t], db, dk[t], 0, 0, 0);  // dK'^T[d][key]
      }
    }
    if (okk) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int d0 = t * 16 + 4 * g;
        float k4[4] = {dk[t][0], dk[t][1], dk[t][2], dk[t][3]};
        float v4[4] = {dv[t][0], dv[t][1], dv[t][2], dv[t][3]};
        rope4_inv(k4, rot, fk, d0, 1.f);  // dk = R^T dK'
        bf16* dst = dqkv + (qrow0 + (int64_t)fk * qfs) * QKV + h * DH + d0;
        store4b(dst + INNER, k4);
        store4b(dst + 2 * INNER, v4);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------- backward, fused (round 5)
// One pass over a (pixel, head) for F > 16 (video_net.py:426-452 differentiated): the two-kernel
// backward above read q, k, v and dO twice, formed S, dP and exp twice and wrote D through HBM; here one wave reads
// q, k, v, dO and O once and forms P and dS once per score tile.  Orientation S[q][key] (A = Q' rows, B = K' rows):
// the MFMA D layout of P and dS (query = 4g + r, key = lane) is directly the B operand of dV^T = dO^T P and
// dK'^T = Q'^T dS through the k-slot map over a query-tile pair (pack_kslot / tr_pair, as the dk / dv kernel), and
// dS reaches the dQ product dQ'^T = K'^T dS^T through a 16 x 16 bf16 LDS tile read back transposed.  Key-tile pairs
// outer (dK / dV of the pair in registers, stored after the pair), query tiles inner, dQ' of every query tile in
// registers for the pixel (2 NT accumulators).  D_i = dO_i . O_i from the forward's output.
// Per wave an LDS region (tfb_wave_bytes): Q' and dO rows of the pixel, the current K' pair (then two dS^T tiles), L, D;
// 64-B rows with 16-B chunk c at c ^ ((row >> 1) & 3): the row-fragment reads, the transposed k-slot reads and the
// staging stores are bank-conflict free (tools/lds_banks.py model).  Rows past the F staged ones are read only against
// P = dS = 0 (padded queries: L = 1e30; padded keys: -inf mask); they fall into the next region's finite rows.
// At F = 120 a block takes 75 KiB: two blocks per CU.
// Rel-pos bias gradient by diagonal d = kt - qt (offset n = 16 d + lane - 4g - r): |d| <= ND in per-(r, d) registers;
// beyond, when the host has checked that every offset there falls in the one saturated bucket per sign (num_buckets 32,
// max_distance 32: |n| >= 27), one accumulator per sign, attributed to offset +-(F - 1) (same bucket, same dtable).
// Grid (4 * TFB_NB, B): block L -> head pair L & 3 and pixel-pair stream L >> 2; its 4 waves are the 2 pixels x the 2
// heads, so the two 64-B head halves of every 128-B qkv / dO / O line are read by one CU at about the same time (the
// first form, one head per block with the 8 heads' blocks on one XCD, fetched 1.5x the algorithmic bytes).
// Measured and removed (round 5, profiles/r5f_*): the next key pair's K / V rows loaded at its start instead of during
// the current pair, a 32 x 32 score block in three phases (192x288, F = 120: 9.6 vs 8.9 ms tile by tile), and
// wave-scope fences around the score loop's LDS round trips -- all within the spread or slower.
// A wave's LDS operations execute in issue order (no s_waitcnt is needed between a ds_write and a later ds_read of the
// same address), and the compiler keeps may-aliasing LDS accesses in program order; the score loop's round trips
// (K' rows -> transposed reads, dS^T tiles -> transposed reads -> the next tile's stores) therefore need no fence,
// and without one the compiler can issue the next tile's reads ahead of the current tile's MFMAs.
constexpr int TFB_NB = 128;
template <typename K>
static void allow_smem(K kernel, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}  // pixel-group streams (blocks) per (sample, head) = cesm_tflash_nblk
__host__ __device__ constexpr int tfb_rq(int F) { return (F + 3) & ~3; }
__host__ __device__ constexpr int tfb_wave_bytes(int F, int NT) {
  return ((2 * tfb_rq(F) * 64 + 32 * 64 + 2 * 64 * NT) + 255) & ~255;
}
// block LDS: the two heads' bias tables (one copy each, 32 NT floats), the RoPE rows of frames 16 a (NT x 32 floats),
// 4 wave regions
static size_t tfb_smem(int F, int NT) { return (size_t)(3 * 32 * NT + 16 * TF_RBS) * 4 + 4 * (size_t)tfb_wave_bytes(F, NT); }
__device__ __forceinline__ void rope4_cs(float* v, const float* cs, float scale) {  // R^T of two pairs, times scale
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const float c = cs[2 * u], s = cs[2 * u + 1];
    const float a = v[2 * u], b = v[2 * u + 1];
    v[2 * u] = (a * c + b * s) * scale;
    v[2 * u + 1] = (b * c - a * s) * scale;
  }
}

template <int NT, int ND>
__global__ __launch_bounds__(256, 2) void tflash_bwd_fused_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ bias, const float* __restrict__ rotg,
    bf16* __restrict__ dqkv, float* __restrict__ part, int F, int HW, float scale, int pm) {
  constexpr int NP = (NT + 1) / 2;
  constexpr int NDG = 2 * ND + 1;    // exact diagonals d = kt - qt in [-ND, ND]
  constexpr bool SAT = ND < NT - 1;  // diagonals beyond: one accumulator per sign
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* rtab = smem;  // [NT][16][2]: RoPE (cos, sin) of frame 16 a
  float* rbase = smem + 3 * 32 * NT;  // [16][TF_RBS]: RoPE (cos, sin) of frames 0 .. 15
  // [2][32 NT]: the block's two heads' bias(n) (log2 units) at k = 16 NT - n (rows = queries: n = key - query)
  float* btabs = smem + 32 * NT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // block = (head pair, pixel-pair stream); wave = (pixel wid >> 1, head of the pair wid & 1): the two waves of a
  // pixel read the two 64-B halves of the same 128-B qkv / dO / O lines at the same time (one HBM fetch per line)
  const int L = blockIdx.x, hp = L & 3, kblk = L >> 2;
  const int h = 2 * hp + (wid & 1);
  const int b = blockIdx.y;
  for (int e = tid; e < 32 * NT; e += 256) rtab[e] = rotg[(e >> 5) * 16 * 32 + (e & 31)];
  for (int e = tid; e < 16 * 32; e += 256)
    rbase[(e >> 5) * TF_RBS + (e & 31)] = e < F * 32 ? rotg[e] : 0.f;  // frames past F (F < 16): 0
  for (int e = tid; e < 2 * 32 * NT; e += 256) {
    const int hh = 2 * hp + e / (32 * NT), n = 16 * NT - e % (32 * NT);
    float v = 0.f;
    if (n > -F && n < F) {
      const int i = n < 0 ? -n : 0, j = i + n;
      v = bias[((int64_t)hh * F + i) * F + j] * LOG2E;
    }
    btabs[e] = v;
  }
  const float* btab = btabs + (wid & 1) * 32 * NT;
  const int RQ = tfb_rq(F);
  char* Qs = reinterpret_cast<char*>(smem + 3 * 32 * NT + 16 * TF_RBS) + wid * tfb_wave_bytes(F, NT);
  char* Os = Qs + RQ * 64;
  char* Ks = Os + RQ * 64;
  // the two dS^T tiles live in the K' rows: those are read (into the dQ A fragments) before the pair's first store
  char* Tt = Ks;
  float* Ls = reinterpret_cast<float*>(Ks + 32 * 64);
  float* Ds = Ls + 16 * NT;
  for (int e = F + lane; e < 16 * NT; e += 64) {  // padded query rows: P = 0 (and so dS = 0)
    Ls[e] = TF_LSE_PAD;
    Ds[e] = 0.f;
  }
  __syncthreads();
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  const int lr = lane & 15, g = lane >> 4, q_ = (lane >> 2) & 3, p_ = lane & 3;
  // row fragment (row lr of a 16-row tile, chunk g), transposed k-slot reads (rows 4g + q_ (+16), 8-B unit p_ of the
  // 16 columns c0 = 16 t), the dS^T tile's store (row lr, 8-B unit g) and transposed read (row 4g + q_, unit p_)
  const int frag = lr * 64 + ((g ^ ((lr >> 1) & 3)) << 4);
  const int trrow = 4 * g + q_;
  int tro[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) tro[t] = trrow * 64 + (((2 * t + (p_ >> 1)) ^ ((trrow >> 1) & 3)) << 4) + (p_ & 1) * 8;
  const int tto = lr * 32 + ((g ^ ((lr >> 2) & 3)) << 3);
  const int tti = trrow * 32 + ((p_ ^ g) << 3);
  auto trp = [&](const char* base, int s, int t) -> bf16x8 {
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(base + s * 2048 + tro[t]));
    const s16x4 c = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(base + s * 2048 + 1024 + tro[t]));
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[j] = __builtin_bit_cast(bf16, (short)a[j]);
      r[4 + j] = __builtin_bit_cast(bf16, (short)c[j]);
    }
    return r;
  };
  const float* bl0 = btab + 4 * g - lr + 16 * NT;  // + 16 (qt - kt) + r: bias of (query 16 qt + 4g + r, key 16 kt + lr)
  // RoPE of frame 16 a + lr by angle addition: the (cos, sin) of frame lr (rbase) composed with the row of frame 16 a
  // (rtab), both block tables in LDS.  (Read per use from the global table, each coefficient load waited behind the
  // wave's earlier stores -- vmcnt counts loads and stores in order -- and the first version of this kernel stalled.)
  auto compose = [](const float* base, f32x4 tile, float* cs, int npairs_off) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float cb = base[npairs_off + 2 * u], sb = base[npairs_off + 2 * u + 1];
      const float ct = tile[2 * u], st = tile[2 * u + 1];
      cs[npairs_off + 2 * u] = cb * ct - sb * st;
      cs[npairs_off + 2 * u + 1] = sb * ct + cb * st;
    }
  };
  const float kmask = 16 * (NT - 1) + lr < F ? 0.f : -INFINITY;  // keys of the last key tile past F

  float dba[4][NDG];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < NDG; ++c) dba[r][c] = 0.f;
  float dsp = 0.f, dsn = 0.f;
  const int ngroups = (HW + 1) / 2;
  const int qfs = pm ? 1 : HW;
  const int fs_qkv = qfs * QKV * 2, fs_io = HW * INNER * 2;  // 16 rows < 2^31 B: checked on the host
  const int lo_qkv = lr * fs_qkv + h * DH * 2 + g * 16, lo_io = lr * fs_io + h * DH * 2 + g * 16;

  for (int gp = kblk; gp < ngroups; gp += TFB_NB) {
    const int p = gp * 2 + (wid >> 1);
    if (p >= HW) break;  // wave-uniform
    const int64_t row0 = (int64_t)b * F * HW + p;
    const int64_t qrow0 = pm ? ((int64_t)b * HW + p) * F : row0;
    // per-pixel opaque copies of the bias / RoPE-row bases: as loop invariants the compiler hoists every per-(tile,
    // lane) bias vector and RoPE row out of the pixel loop (> 100 VGPRs at NT = 8) and spills
    const float* bl = bl0 + opaque_zero();
    const float* rt = rtab + opaque_zero();
    const float* rb = rbase + lr * TF_RBS + opaque_zero();
    auto cs8 = [&](int a, float* cs) {  // pairs 4g .. 4g + 3 of frame 16 a + lr
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(rb + 8 * g), b1 = *reinterpret_cast<const f32x4*>(rb + 8 * g + 4);
      const float cb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      compose(cb, *reinterpret_cast<const f32x4*>(rt + a * 32 + 8 * g), cs, 0);
      compose(cb, *reinterpret_cast<const f32x4*>(rt + a * 32 + 8 * g + 4), cs, 4);
    };
    auto cs4 = [&](int a, int t, float* cs) {  // pairs 8t + 2g, +1 of frame 16 a + lr
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(rb + (8 * t + 2 * g) * 2);
      const float cb[4] = {b0[0], b0[1], b0[2], b0[3]};
      compose(cb, *reinterpret_cast<const f32x4*>(rt + a * 32 + (8 * t + 2 * g) * 2), cs, 0);
    };
    bf16x8 kraw[2], vraw[2];
    auto ldkv = [&](int sk) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int kt = 2 * sk + u;
        const auto rs = tile_rsrc(qkv + (qrow0 + (int64_t)kt * 16 * qfs) * QKV, F - kt * 16, (int64_t)fs_qkv, QKV * 2);
        kraw[u] = buf_ld16(rs, lo_qkv + INNER * 2);  // frames >= F: zeros
        vraw[u] = buf_ld16(rs, lo_qkv + 2 * INNER * 2);
      }
    };
    ldkv(0);
    wsync();  // the previous pixel's reads of the region done
    // ---- stage Q' = scale R q and dO rows, L and D = dO . O of the pixel's queries: every load issued first (rows past
    // F read as zeros), then branch-free stores -- Q' tiles before dO tiles, so the zero rows the last Q' tile writes
    // past the RQ staged ones (into the dO rows) are overwritten; the dO tile's land in the K' rows, staged later
    const float* lsep = lse + (((int64_t)b * NH + h) * HW + p) * F;
    bf16x8 qr[NT], dr[NT], orw[NT];
    float lq[NT];
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) {
      const int nq = F - qt * 16;
      const auto rq = tile_rsrc(qkv + (qrow0 + (int64_t)qt * 16 * qfs) * QKV, nq, (int64_t)fs_qkv, QKV * 2);
      const auto rd = tile_rsrc(dout + (row0 + (int64_t)qt * 16 * HW) * INNER, nq, (int64_t)fs_io, INNER * 2);
      const auto ro = tile_rsrc(o + (row0 + (int64_t)qt * 16 * HW) * INNER, nq, (int64_t)fs_io, INNER * 2);
      qr[qt] = buf_ld16(rq, lo_qkv);
      dr[qt] = buf_ld16(rd, lo_io);
      orw[qt] = buf_ld16(ro, lo_io);
      const int f = qt * 16 + lr;
      lq[qt] = lsep[f < F ? f : 0];
    }
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) {
      float cs[8];
      cs8(qt, cs);
      *reinterpret_cast<bf16x8*>(Qs + qt * 1024 + frag) = rope8(qr[qt], cs, scale);
    }
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) {
      *reinterpret_cast<bf16x8*>(Os + qt * 1024 + frag) = dr[qt];
      float Do = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) Do = fmaf((float)dr[qt][e], (float)orw[qt][e], Do);
      const float D = grp4_sum(Do);
      const int f = qt * 16 + lr;  // the 4 lanes of a row store the same values
      Ls[f] = f < F ? lq[qt] : TF_LSE_PAD;
      Ds[f] = f < F ? D : 0.f;
    }
    f32x4 dq[NT][2];
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) dq[qt][0] = dq[qt][1] = z4;

#pragma unroll
    for (int sk = 0; sk < NP; ++sk) {
      // K' rows of the key pair: B fragments of S, staged for the transposed reads of the dQ product
      bf16x8 kb[2], vb[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float cs[8];
        cs8(2 * sk + u < NT ? 2 * sk + u : 0, cs);
        kb[u] = rope8(kraw[u], cs, 1.f);  // keys >= F: zeros
        vb[u] = vraw[u];
        *reinterpret_cast<bf16x8*>(Ks + u * 1024 + frag) = kb[u];
      }
      if (sk + 1 < NP) ldkv(sk + 1);
      const bf16x8 ka[2] = {trp(Ks, 0, 0), trp(Ks, 0, 1)};  // K'^T[d][keys of the pair]
      f32x4 dk[2][2], dv[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) dk[u][0] = dk[u][1] = dv[u][0] = dv[u][1] = z4;
#pragma unroll
      for (int sq = 0; sq < NP; ++sq) {
        // P and dS of the pair block as bf16 k-slot B fragments per key tile (slots j < 4: query tile 2 sq, j >= 4: 2 sq + 1)
        bf16x8 pb[2], sb[2];
#pragma unroll
        for (int uq = 0; uq < 2; ++uq) {
          const int qt = 2 * sq + uq;
          if (qt >= NT) {
#pragma unroll
            for (int uk = 0; uk < 2; ++uk)
#pragma unroll
              for (int r = 0; r < 4; ++r) pb[uk][4 * uq + r] = sb[uk][4 * uq + r] = (bf16)0.f;
            continue;
          }
          const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + qt * 1024 + frag);
          const bf16x8 da = *reinterpret_cast<const bf16x8*>(Os + qt * 1024 + frag);
          const f32x4 Lq = *reinterpret_cast<const f32x4*>(Ls + qt * 16 + 4 * g);
          const f32x4 Dq = *reinterpret_cast<const f32x4*>(Ds + qt * 16 + 4 * g);
#pragma unroll
          for (int uk = 0; uk < 2; ++uk) {
            const int kt = 2 * sk + uk;
            float sv[4];
            if (kt < NT) {
              const f32x4 sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kb[uk], z4, 0, 0, 0);  // S'[q][key]
              const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, vb[uk], z4, 0, 0, 0);  // dP[q][key]
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                float x = fmaf(sc[r], LOG2E, bl[16 * (qt - kt) + r]) - Lq[r];
                if (kt == NT - 1) x += kmask;
                const float pp = __builtin_amdgcn_exp2f(x);
                const float ds = pp * (dp[r] - Dq[r]);
                pb[uk][4 * uq + r] = (bf16)pp;
                sv[r] = ds;
                const int dd = kt - qt;
                if (dd >= -ND && dd <= ND) dba[r][dd + ND] += ds;
                else if (dd > 0) dsp += ds;
                else dsn += ds;
              }
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                pb[uk][4 * uq + r] = (bf16)0.f;
                sv[r] = 0.f;
              }
            }
            const bf16x4 t4 = {(bf16)sv[0], (bf16)sv[1], (bf16)sv[2], (bf16)sv[3]};
#pragma unroll
            for (int r = 0; r < 4; ++r) sb[uk][4 * uq + r] = t4[r];
            *reinterpret_cast<bf16x4*>(Tt + (uq * 2 + uk) * 512 + tto) = t4;  // dS^T[key = lane][q = 4g .. 4g + 3]
          }
          // dQ'^T[d][q] += K'^T[d][keys] dS^T[keys][q] over the pair's 32 keys
          const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(Tt + (uq * 2) * 512 + tti));
          const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(Tt + (uq * 2 + 1) * 512 + tti));
          bf16x8 bsd;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            bsd[j] = __builtin_bit_cast(bf16, (short)t0[j]);
            bsd[4 + j] = __builtin_bit_cast(bf16, (short)t1[j]);
          }
#pragma unroll
          for (int t = 0; t < 2; ++t) dq[qt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[t], bsd, dq[qt][t], 0, 0, 0);
        }
        // dV^T[d][key] += dO^T[d][q] P[q][key], dK'^T[d][key] += Q'^T[d][q] dS[q][key] over the query pair's 32 rows
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 dta = trp(Os, sq, t), qta = trp(Qs, sq, t);
#pragma unroll
          for (int uk = 0; uk < 2; ++uk) {
            if (2 * sk + uk >= NT) continue;
            dv[uk][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dta, pb[uk], dv[uk][t], 0, 0, 0);
            dk[uk][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qta, sb[uk], dk[uk][t], 0, 0, 0);
          }
        }
      }
      // dk = R^T dK', dv of the pair's keys (rows >= F dropped by the resource)
#pragma unroll
      for (int uk = 0; uk < 2; ++uk) {
        const int kt = 2 * sk + uk;
        if (kt >= NT) continue;
        const auto rs = tile_rsrc(dqkv + (qrow0 + (int64_t)kt * 16 * qfs) * QKV, F - kt * 16,
                                  (int64_t)fs_qkv, QKV * 2);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int d0 = t * 16 + 4 * g;
          float k4[4] = {dk[uk][t][0], dk[uk][t][1], dk[uk][t][2], dk[uk][t][3]};
          const float v4[4] = {dv[uk][t][0], dv[uk][t][1], dv[uk][t][2], dv[uk][t][3]};
          float cs[4];
          cs4(kt, t, cs);
          rope4_cs(k4, cs, 1.f);
          buf_st4b(rs, lr * fs_qkv + (INNER + h * DH + d0) * 2, k4);
          buf_st4b(rs, lr * fs_qkv + (2 * INNER + h * DH + d0) * 2, v4);
        }
      }
    }
    // dq = scale R^T dQ'
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) {
      const auto rs = tile_rsrc(dqkv + (qrow0 + (int64_t)qt * 16 * qfs) * QKV, F - qt * 16,
                                (int64_t)fs_qkv, QKV * 2);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int d0 = t * 16 + 4 * g;
        float v4[4] = {dq[qt][t][0], dq[qt][t][1], dq[qt][t][2], dq[qt][t][3]};
        float cs[4];
        cs4(qt, t, cs);
        rope4_cs(v4, cs, scale);
        buf_st4b(rs, lr * fs_qkv + (h * DH + d0) * 2, v4);
      }
    }
  }
  // ---- rel-pos bias partials of the block: offset n = 16 d + l - 4 gg - r of lane (gg, l), register r, diagonal d;
  // each lane sums the offsets n = lane + 64 j - (F - 1) over (d, gg, r) in a fixed order, the block its 4 waves in order
  wsync();
  float* stg = reinterpret_cast<float*>(Qs);  // NDG * 4 rows of 64 floats (<= the wave's Q', dO and K' rows)
#pragma unroll
  for (int c = 0; c < NDG; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) stg[(c * 4 + r) * 64 + lane] = dba[r][c];
  const float tp = SAT ? wave_sum(dsp) : 0.f, tn = SAT ? wave_sum(dsn) : 0.f;
  wsync();
  float* wsum = reinterpret_cast<float*>(Ks);  // 256 floats (after the sums: the staged rows may reach into Ks)
  float asum[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = lane + 64 * j - (F - 1);
    float a = 0.f;
    if (n < F) {
#pragma nounroll
      for (int c = 0; c < NDG; ++c)
#pragma nounroll
        for (int gg = 0; gg < 4; ++gg)
#pragma nounroll
          for (int r = 0; r < 4; ++r) {
            const int l = n - 16 * (c - ND) + 4 * gg + r;
            if (l >= 0 && l < 16) a += stg[(c * 4 + r) * 64 + gg * 16 + l];
          }
      if (SAT && n == F - 1) a += tp;
      if (SAT && n == -(F - 1)) a += tn;
    }
    asum[j] = a;
  }
  wsync();
#pragma unroll
  for (int j = 0; j < 4; ++j) wsum[lane + 64 * j] = asum[j];
  __syncthreads();
  if (part) {  // per head of the pair: its two waves (pixels) in order
    const float* w0 = reinterpret_cast<const float*>(reinterpret_cast<char*>(smem + 3 * 32 * NT + 16 * TF_RBS) + 2 * (tfb_rq(F) * 64));
    const int WB = tfb_wave_bytes(F, NT) / 4;
#pragma clang loop vectorize(disable)  // (the tflash sources stay free of packed fp32: tests/test_isa_guard.py)
    for (int e = tid; e < 2 * (2 * F - 1); e += 256) {
      const int u = e / (2 * F - 1), n = e - u * (2 * F - 1);
      part[((int64_t)(b * NH + 2 * hp + u) * TFB_NB + kblk) * (2 * F - 1) + n] = w0[u * WB + n] + w0[(2 + u) * WB + n];
    }
  }
}

// dtable[bucket][h] (+)= sum over partials and offsets n with bucket(n) of part[(b*8 + h)][blk][n + F - 1]
__device__ int tf_bucket(int rel, int num_buckets, int max_distance) {  // relpos_bucket of attn.hip
  int n = -rel;
  const int nb = num_buckets / 2;
  int ret = n < 0 ? nb : 0;
  n = n < 0 ? -n : n;
  const int max_exact = nb / 2;
  if (n < max_exact) return ret + n;
  const float lg = logf((float)n / (float)max_exact) / logf((float)max_distance / (float)max_exact) *
                   (float)(nb - max_exact);
  int large = max_exact + (int)lg;
  if (large > nb - 1) large = nb - 1;
  return ret + large;
}
// stage 1: off[h][n] = sum over samples and blocks (block per (h, n), fixed order)
__global__ void tf_dbias_off_kernel(const float* __restrict__ part, float* __restrict__ off, int nblk, int B, int F) {
  const int h = blockIdx.y, e = blockIdx.x;
  const int NO = 2 * F - 1;
  float s = 0.f;
  for (int k = threadIdx.x; k < B * nblk; k += 256) {
    const int bb = k / nblk, kk = k - bb * nblk;
    s += part[((int64_t)(bb * NH + h) * nblk + kk) * NO + e];
  }
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) off[h * NO + e] = red[0] + red[1] + red[2] + red[3];
}
// stage 2: dtable[bucket][h] (+)= sum of off[h][n] over the offsets of that bucket
__global__ void tf_dtable_kernel(const float* __restrict__ off, float* __restrict__ dtable, int F, int num_buckets,
                                 int max_distance, int accumulate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= num_buckets * NH) return;
  const int bk = t / NH, h = t % NH;
  float s = 0.f;
  for (int n = -(F - 1); n < F; ++n)
    if (tf_bucket(n, num_buckets, max_distance) == bk) s += off[h * (2 * F - 1) + n + F - 1];
  dtable[t] = accumulate ? dtable[t] + s : s;
}

}  // namespace

// which backward cesm_tflash_bwd runs: the one-pass fused kernel (round 5) for every window of F >= 8 frames, the
// two-kernel form below that (its D = sum P dP keeps the F = 1 rel-pos bias gradient exactly 0, where D = dO . O from
// the bf16 O would leave a rounding residue).  Round 6 removed the other dq kernels: the per-wave dq kernel (slower
// in the F = 120 step: 232.5-233.0 vs 229.9-230.0 ms, profiles/r4c13_env_ab.txt), the single-pass D = dO . O kernel
// for small levels, and the CESM_TF_FUSED=0 switch back to the two-kernel form at F >= 8.
enum TfDq { TF_DQ_BLOCK, TF_FUSED };
// host copy of tf_bucket (relpos_bucket): the fused backward's saturated-diagonal check
static int tf_bucket_host(int rel, int num_buckets, int max_distance) {
  int n = -rel;
  const int nb = num_buckets / 2;
  int ret = n < 0 ? nb : 0;
  n = n < 0 ? -n : n;
  const int max_exact = nb / 2;
  if (n < max_exact) return ret + n;
  const float lg = logf((float)n / (float)max_exact) / logf((float)max_distance / (float)max_exact) *
                   (float)(nb - max_exact);
  int large = max_exact + (int)lg;
  if (large > nb - 1) large = nb - 1;
  return ret + large;
}
// exact bias-gradient diagonals per side the fused backward needs: the smallest nd whose beyond-diagonals' offsets
// (|n| >= 16 nd + 1, with a margin of 2 for float rounding of the bucket logarithm) all share the bucket of +-(F - 1)
static int tfb_nd(int F, int nt, int num_buckets, int max_distance) {
  const int bp = tf_bucket_host(F - 1, num_buckets, max_distance), bn = tf_bucket_host(-(F - 1), num_buckets, max_distance);
  for (int nd = 0; nd < nt - 1; ++nd) {
    bool ok = true;
    for (int n = std::max(1, 16 * nd - 1); n < F && ok; ++n)
      ok = tf_bucket_host(n, num_buckets, max_distance) == bp && tf_bucket_host(-n, num_buckets, max_distance) == bn;
    if (ok) return nd;
  }
  return nt - 1;
}
static TfDq tf_dq_kind(int nt, int F) { return nt >= 2 || F >= 8 ? TF_FUSED : TF_DQ_BLOCK; }

extern "C" {

// name of the dq kernel cesm_tflash_bwd runs for (F, HW) with frame-major qkv (host-only query; "invalid" when F
// is unsupported)
const char* cesm_tflash_bwd_variant(int F, int HW) {
  static const char* fused[9] = {"", "tflash_bwd_fused_kernel<1>", "tflash_bwd_fused_kernel<2>", "tflash_bwd_fused_kernel<3>",
                                 "tflash_bwd_fused_kernel<4>", "tflash_bwd_fused_kernel<5>", "tflash_bwd_fused_kernel<6>",
                                 "tflash_bwd_fused_kernel<7>", "tflash_bwd_fused_kernel<8>"};
  if (F < 1 || F > 16 * TF_MAXT || HW < 1) return "invalid";
  const int nt = (F + 15) / 16;
  return tf_dq_kind(nt, F) == TF_FUSED ? fused[nt] : "tflash_bwd_q_kernel<1>";
}

// supported windows of the MFMA temporal-attention core (bf16)
int cesm_tflash_supported(int F) { return F >= 1 && F <= 16 * TF_MAXT; }

// blocks per (sample, head) of cesm_tflash_bwd's dq kernel (its dbias partial rows)
int cesm_tflash_nblk(int HW) { return (void)HW, TFB_NB; }

// forward: qkv [B*F*HW][768] bf16 -> out [B*F*HW][256] bf16, lse [B][8][HW][F] (log2 units, nullable);
// bias [8][F][F] (expanded rel-pos bias), rot [F][16][2].  qkv_pixel_major (F > 16 only): qkv rows ordered
// [B][HW][F] (a pixel's frames adjacent) instead of [B][F][HW]; out stays [B][F][HW].
int cesm_tflash_fwd(const void* qkv, const float* bias, const float* rot, void* out, float* lse, int B, int F, int HW,
                    float scale, int qkv_pixel_major, hipStream_t stream) {
  if (!cesm_tflash_supported(F) || B < 1 || HW < 1) return CESM_EUNSUPPORTED;
  const int nt = (F + 15) / 16;
  const int pm = qkv_pixel_major ? 1 : 0;
  if (pm && nt < 2) return CESM_EUNSUPPORTED;
  if ((int64_t)16 * HW * (pm ? INNER : QKV) * 2 >= (1ll << 31)) return CESM_EUNSUPPORTED;  // 32-bit lane offsets
  dim3 grid(tf_grid_x(HW), B);
#define TFF(N) \
  tflash_fwd2_kernel<N><<<grid, 256, 0, stream>>>((const bf16*)qkv, bias, rot, (bf16*)out, lse, F, HW, scale, pm)
  switch (nt) {
    case 1: TFF(1); break;
    case 2: TFF(2); break;
    case 3: TFF(3); break;
    case 4: TFF(4); break;
    case 5: TFF(5); break;
    case 6: TFF(6); break;
    case 7: TFF(7); break;
    case 8: TFF(8); break;
    default: return CESM_EUNSUPPORTED;
  }
#undef TFF
  return cesm_launch_status();
}

// backward: dqkv [B*F*HW][768] (every channel written; in qkv's row order), from qkv, the forward's o and lse, and
// dout [..][256] (frame-major);
// dtable (+)= the rel-pos table gradient (nullable).  Workspaces: dbuf B*8*HW*F floats, part
// B*8*nblk*(2F-1) floats (nblk = cesm_tflash_nblk(HW)), off 8*(2F-1) floats.
int cesm_tflash_bwd(const void* qkv, const void* o, const void* dout, const float* lse, const float* bias,
                    const float* rot, void* dqkv, float* dtable, float* dbuf, float* part, float* off, int B, int F,
                    int HW, float scale, int num_buckets, int max_distance, int accumulate, int qkv_pixel_major,
                    hipStream_t stream) {
  if (!cesm_tflash_supported(F) || B < 1 || HW < 1) return CESM_EUNSUPPORTED;
  const int nt = (F + 15) / 16;
  const int pm = qkv_pixel_major ? 1 : 0;
  if (pm && (nt < 2 || (int64_t)16 * HW * INNER * 2 >= (1ll << 31))) return CESM_EUNSUPPORTED;
  const int nblk = cesm_tflash_nblk(HW);
  dim3 gq(nblk, B * NH), gk(tf_grid_x(HW), B);
  const TfDq kind = tf_dq_kind(nt, F);
  if (kind == TF_FUSED) {
    if ((int64_t)16 * (pm ? 1 : HW) * QKV * 2 >= (1ll << 31))
      return CESM_EUNSUPPORTED;  // 32-bit lane offsets of a 16-row tile
    const int nd = tfb_nd(F, nt, num_buckets, max_distance);
    const size_t sm = tfb_smem(F, nt);
    dim3 gf(4 * TFB_NB, B);
    float* pt = dtable ? part : nullptr;
#define TFU(N, D)                                                                                                    \
  {                                                                                                                  \
    allow_smem(tflash_bwd_fused_kernel<N, D>, sm);                                                                   \
    tflash_bwd_fused_kernel<N, D><<<gf, 256, sm, stream>>>((const bf16*)qkv, (const bf16*)o, (const bf16*)dout, lse, \
                                                           bias, rot, (bf16*)dqkv, pt, F, HW, scale, pm);            \
  }
#define TFUN(N)                           \
  if (N >= 4 && nd <= 2) TFU(N, (N >= 4 ? 2 : N - 1)) \
  else TFU(N, N - 1)
    switch (nt) {
      case 1: TFU(1, 0); break;
      case 2: TFU(2, 1); break;
      case 3: TFU(3, 2); break;
      case 4: TFUN(4); break;
      case 5: TFUN(5); break;
      case 6: TFUN(6); break;
      case 7: TFUN(7); break;
      case 8: TFUN(8); break;
      default: return CESM_EUNSUPPORTED;
    }
#undef TFUN
#undef TFU
  } else {  // F < 8: one 16-frame tile
    tflash_bwd_q_kernel<1><<<gq, 64, 0, stream>>>((const bf16*)qkv, (const bf16*)o, (const bf16*)dout, lse, bias, rot,
                                                 (bf16*)dqkv, dbuf, part, F, HW, scale, pm);
    tflash_bwd_kv_kernel<1><<<gk, 256, 0, stream>>>((const bf16*)qkv, (const bf16*)dout, lse, dbuf, bias, rot,
                                                   (bf16*)dqkv, F, HW, scale, pm);
  }
  if (dtable) {
    tf_dbias_off_kernel<<<dim3(2 * F - 1, NH), 256, 0, stream>>>(part, off, nblk, B, F);
    tf_dtable_kernel<<<(unsigned)cdiv(num_buckets * NH, 64), 64, 0, stream>>>(off, dtable, F, num_buckets,
                                                                               max_distance, accumulate);
  }
  return cesm_launch_status();
}

}  // extern "C"
