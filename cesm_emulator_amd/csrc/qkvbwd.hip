// Backward of the 768-channel qkv projection (1x1 conv / Linear without bias) with dqkv read ONCE (round 6,
// VERDICT r5 item 4): video_net.py:380-381 (to_qkv of the temporal Attention) and :322-323 (SpatialLinearAttention),
// differentiated --
//
//   dX[m][c] = sum_n dY[m][n] W[n][c]          (dgrad: the LN output's gradient)
//   dW[n][c] = sum_m dY[m][n] X[m][c]          (wgrad)
//
// with dY = dqkv [M][N = 768] bf16, X = the LN output [M][C] bf16, W = to_qkv.weight [N][C].  The unfused path read
// dqkv twice (a 1x1 MFMA GEMM for dX, then a wide weight-gradient GEMM for dW): at level 0 of the decadal window
// (192 x 288 x 120 pixels) that is 10.2 GB per read.
//
// Persistent blocks of 8 waves (one per CU), each owning a 64-channel slice of C and a stream of 64-pixel tiles.  A
// tile's dY rows go through LDS in six 128-channel chunks (16 KiB each; a ring of QB_NS stages filled by LDS-DMA,
// QB_NS - 1 chunks in flight); the slice's W^T rows (96 KiB) stay in LDS.  Per chunk every wave does
//   wgrad: its 16 n rows of the chunk x the slice's 64 c, K = the tile's 64 pixels (8 MFMAs; A = dY^T and B = X^T by
//          the hardware transpose read, the X^T fragments read once per tile);
//   dgrad: D[c][px] for its c tile and two pixel tiles, K = the chunk's 128 n (8 MFMAs; A = W^T rows, B = dY rows).
// (The first form read the W^T fragments from L2 one chunk ahead: every chunk then waited out an L2 round trip,
// 2.8 TB/s at the decadal window's level 0 -- slower than the two GEMMs it replaces.)
// dW accumulators for all 768 n x 64 c stay in registers for the whole kernel (wave w: n rows 128 k + 16 w of every
// chunk k: 24 tiles, 96 VGPRs) and are written once as a per-block fp32 slab, summed over blocks in a fixed order
// (qkv_bwd_reduce_kernel): the result is bit-repeatable.
//
// Roofline: HBM.  Per pixel 2 N + 4 C bytes (dY, X in, dX out) for 4 N C FLOP: at N = 768, C = 64 about 1.8 KB and
// 197 kFLOP, i.e. 110 FLOP/B against the chip's ~310 (2.5 PF/s / 8 TB/s).
#include "common.h"
#include "cesm_hip.h"

namespace {

constexpr int QB_BP = 64;                   // pixels per tile
constexpr int QB_CN = 128;                  // qkv channels per LDS chunk
constexpr int QB_NS = 3;                    // chunk stages in the ring
constexpr int QB_STAGE = QB_BP * QB_CN * 2;  // 16 KiB
constexpr int QB_XT = QB_BP * 64 * 2;        // 8 KiB: a tile's X slice
constexpr int QB_N = 768;
constexpr int QB_WT = 64 * QB_N * 2;         // 96 KiB: the slice's W^T rows, resident
constexpr int QB_LDS = QB_WT + QB_NS * QB_STAGE + QB_XT + 1024;  // + a 1-KiB sink for the balancing DMA pieces
static_assert(QB_LDS <= 160 * 1024, "qkv_bwd LDS");

// 16-B slot swizzles (tools/qkv_lds_banks.py enumerates the LDS bank groups of each read form): dY chunk rows (256 B):
// ds_read_b128 of 16 rows x one chunk and ds_read_b64_tr_b16 of 4 rows x 4 8-B chunks both conflict-free; X rows
// (128 B): the transposed reads conflict-free; W^T rows (1536 B): ds_read_b128 of 16 rows x one chunk conflict-free.
__device__ __forceinline__ int qb_fa(int r) { return ((r & 1) << 3) | ((r & 2) << 1) | (((r >> 3) & 1) << 1); }
__device__ __forceinline__ int qb_fb(int r) { return ((r & 2) << 1) | (((r >> 3) & 1) << 1); }
__device__ __forceinline__ int qb_a_off(int r, int c16) { return r * 256 + ((c16 ^ qb_fa(r)) << 4); }
__device__ __forceinline__ int qb_b_off(int r, int c16) { return r * 128 + ((c16 ^ qb_fb(r)) << 4); }
__device__ __forceinline__ int qb_w_off(int r, int c16) { return r * (QB_N * 2) + ((c16 ^ (r & 15)) << 4); }

typedef __attribute__((address_space(3))) void* lds_vptr;
typedef unsigned int qb_u32x2 __attribute__((ext_vector_type(2)));

// grid: nsl * nstream blocks (nsl = C / 64 slices, nstream a multiple of 8; a stream's slices on one XCD)
template <int NCH>
__global__ __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2))) void qkv_bwd_kernel(
    const bf16* __restrict__ dy, const bf16* __restrict__ x, const bf16* __restrict__ wt, bf16* __restrict__ dx,
    float* __restrict__ slab, int64_t M, int C, int ntiles) {
  constexpr int N = NCH * QB_CN;
  static_assert(N == QB_N, "the resident W^T slice is sized for N = 768");
  __shared__ __attribute__((aligned(1024))) char lds[QB_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int nsl = C / 64;
  const int L = blockIdx.x, jx = L >> 3;
  const int sl = jx % nsl;
  const int stream = (jx / nsl) * 8 + (L & 7);
  const int nstream = (int)(gridDim.x / nsl);
  const int c0 = sl * 64;
  // this block's tiles: stream, stream + nstream, ...; steps = tiles x NCH chunks
  const int my_tiles = stream < ntiles ? (ntiles - 1 - stream) / nstream + 1 : 0;
  const int nsteps = my_tiles * NCH;
  char* ws = lds;                      // [64][N] W^T rows of the slice
  char* ring = lds + QB_WT;            // [QB_NS][QB_STAGE]
  char* xs = ring + QB_NS * QB_STAGE;  // [QB_XT]
  char* sink = xs + QB_XT;
  if (nsteps == 0) {  // a padding stream (fewer tiles than streams): its slab holds zeros
    if (slab) {
      float* out = slab + ((int64_t)sl * nstream + stream) * N * 64;
      for (int e = tid; e < N * 64; e += 512) out[e] = 0.f;
    }
    return;
  }

  // LDS-DMA of step s (tile s / NCH, chunk s % NCH): 2 pieces of the dY chunk per wave + one X piece (chunk 0) or one
  // out-of-range piece into the sink, so every step issues 3 pieces per wave and one counted vmcnt fits every step
  auto issue = [&](int s) {
    if (s >= nsteps) {  // past the last step: 3 sink pieces (zeros), the count stays the same
      const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, 0, 0x00020000);
#pragma unroll
      for (int p = 0; p < 3; ++p) __builtin_amdgcn_raw_ptr_buffer_load_lds(zrs, (lds_vptr)sink, 16, 0, 0, 0, 0);
      return;
    }
    const int k = s / NCH, ch = s - k * NCH;
    const int64_t m0 = (int64_t)(stream + k * nstream) * QB_BP;
    const int rows = M - m0 < QB_BP ? (int)(M - m0) : QB_BP;
    const __amdgpu_buffer_rsrc_t yrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(dy + m0 * N), (short)0, rows * N * 2, 0x00020000);
    char* st = ring + (s % QB_NS) * QB_STAGE;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int q = wid + 8 * p, row = 4 * q + (lane >> 4);
      const int c16 = (lane & 15) ^ qb_fa(row);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yrs, (lds_vptr)(st + q * 1024), 16,
                                               (row * N + ch * QB_CN + c16 * 8) * 2, 0, 0, 0);
    }
    if (ch == 0) {  // uniform
      const __amdgpu_buffer_rsrc_t xrs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(x + m0 * C + c0), (short)0, rows * C * 2 - c0 * 2, 0x00020000);
      const int row = 8 * wid + (lane >> 3);
      const int c16 = (lane & 7) ^ qb_fb(row);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_vptr)(xs + wid * 1024), 16, (row * C + c16 * 8) * 2, 0, 0,
                                               0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yrs, (lds_vptr)sink, 16, 0x7fff8000, 0, 0, 0);  // out of range: zeros
    }
  };

  // prologue: the slice's W^T rows (96 KiB: 12 pieces per wave), then the DMA of steps 0 .. QB_NS - 2
  {
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(wt + (int64_t)c0 * N), (short)0, 64 * N * 2, 0x00020000);
#pragma unroll
    for (int p = 0; p < QB_WT / 1024 / 8; ++p) {
      const int piece = wid + 8 * p;
      const int e16 = piece * 64 + lane, row = e16 / (N / 8), slot = e16 - row * (N / 8);
      const int c16 = (slot & ~15) | ((slot & 15) ^ (row & 15));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_vptr)(ws + piece * 1024), 16, (row * N + c16 * 8) * 2, 0, 0,
                                               0);
    }
  }
#pragma unroll
  for (int s = 0; s < QB_NS - 1; ++s) issue(s);

  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 dwacc[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) dwacc[c][j] = z4;
  const int q = lr >> 2, pp = lr & 3;
  const int ct = wid & 3;    // dgrad c tile
  const int pt0 = wid >> 2;  // dgrad pixel tiles pt0, pt0 + 2

  for (int k = 0; k < my_tiles; ++k) {
    const int64_t m0 = (int64_t)(stream + k * nstream) * QB_BP;
    bf16x8 bx[2][4];  // wgrad B = X^T fragments of the tile (K = pixels), read at chunk 0 (the X buffer is then free)
    f32x4 dxacc[2] = {z4, z4};
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int s = k * NCH + ch;
      // this step's DMA was issued QB_NS - 1 = 2 steps ago; younger: the previous step's DMA (3 pieces) and, after a
      // tile end, its 2 dX stores (at step 0 the W^T pieces are older still)
      static_assert(QB_NS == 3, "the counted vmcnt below assumes one younger DMA step");
      if (ch == 0 && k > 0) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      __syncthreads();  // every wave's pieces of this stage landed; the stage issued next is no longer read
      issue(s + QB_NS - 1);
      const char* st = ring + (s % QB_NS) * QB_STAGE;
      if (ch == 0) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int half = 0; half < 2; ++half) {
              const int r = kk * 32 + lg * 8 + half * 4 + q, c8 = j * 4 + pp;
              const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (LDS_PTR(s16x4))(xs + qb_b_off(r, c8 >> 1) + (c8 & 1) * 8));
#pragma unroll
              for (int e = 0; e < 4; ++e) bx[kk][j][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
            }
      }
      // wgrad: dW[n rows 16 wid.. of chunk ch][c] += dY^T . X over the tile's pixels
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int r = kk * 32 + lg * 8 + half * 4 + q, c8 = wid * 4 + pp;
          const s16x4 v =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(st + qb_a_off(r, c8 >> 1) + (c8 & 1) * 8));
#pragma unroll
          for (int e = 0; e < 4; ++e) af[half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) dwacc[ch][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bx[kk][j], dwacc[ch][j], 0, 0, 0);
      }
      // dgrad: dX^T[c tile ct][pixel tiles pt0, pt0 + 2] += W^T . dY^T over the chunk's 128 n
#pragma unroll
      for (int kn = 0; kn < 4; ++kn) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(ws + qb_w_off(ct * 16 + lr, ch * 16 + kn * 4 + lg));
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int r = (pt0 + 2 * u) * 16 + lr;
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(st + qb_a_off(r, kn * 4 + lg));
          dxacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, dxacc[u], 0, 0, 0);
        }
      }
    }
    // dX of the tile: lane holds c = c0 + 16 ct + 4 lg .. +3 of pixel (pt0 + 2u) * 16 + lr; 8-B stores through a
    // buffer resource over the tile (rows past M: out of range, dropped), always 2 per lane (the counted vmcnt above)
    {
      const int rows = M - m0 < QB_BP ? (int)(M - m0) : QB_BP;
      const __amdgpu_buffer_rsrc_t drs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(dx + m0 * C), (short)0, rows * C * 2, 0x00020000);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int p = (pt0 + 2 * u) * 16 + lr;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)dxacc[u][r];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(qb_u32x2, o), drs, (p * C + c0 + ct * 16 + lg * 4) * 2,
                                              0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // per-block dW slab [N][64] of this slice: slab[(sl * nstream + stream)][n][c]
  if (slab) {
    float* out = slab + ((int64_t)sl * nstream + stream) * N * 64;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(int64_t)(ch * QB_CN + wid * 16 + lg * 4 + r) * 64 + j * 16 + lr] = dwacc[ch][j][r];
  }
}

// dw[n][c] (+)= sum over the slice's nstream slabs (fixed order)
__global__ void qkv_bwd_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw, int N, int C, int nstream,
                                      int accumulate) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)N * C) return;
  const int n = (int)(e / C), c = (int)(e - (int64_t)n * C), sl = c >> 6, cc = c & 63;
  const float* p = slab + ((int64_t)sl * nstream * N + n) * 64 + cc;
  float s = 0.f;
  for (int b = 0; b < nstream; ++b) s += p[(int64_t)b * N * 64];
  dw[e] = accumulate ? dw[e] + s : s;
}

int qkv_bwd_streams(int64_t M, int C) {
  const int64_t ntiles = (M + QB_BP - 1) / QB_BP;
  const int nsl = C / 64;
  int per = cesm_num_cus() / nsl;  // one block per CU over the slices
  if (per < 8) per = 8;
  per = per / 8 * 8;
  const int64_t need = (ntiles + 7) / 8 * 8;
  return (int)(need < per ? need : per);
}

}  // namespace

extern "C" {

// streams (blocks per 64-channel slice) of cesm_qkv_bwd; its slab holds (C / 64) * streams * N * 64 floats
int cesm_qkv_bwd_streams(int64_t M, int N, int C) {
  if (M < 1 || N != 768 || C < 64 || C % 64 || C > 512) return 0;
  return qkv_bwd_streams(M, C);
}

// dy [M][N] bf16 (N = 768), x [M][C] bf16, wt [C][N] bf16 (the weight transposed: wt[c][n] = W[n][c]);
// dx [M][C] bf16 (written); dw [N][C] fp32 (+= if accumulate; nullable: no weight gradient);
// slab (C / 64) * streams * N * 64 floats (streams = cesm_qkv_bwd_streams; nullable when dw is).
int cesm_qkv_bwd(const void* dy, const void* x, const void* wt, void* dx, float* dw, float* slab, int64_t M, int N,
                 int C, int accumulate, hipStream_t stream) {
  const int ns = cesm_qkv_bwd_streams(M, N, C);
  if (ns == 0) return CESM_EUNSUPPORTED;
  if (dw && !slab) return CESM_EINVAL;
  const int64_t ntiles = (M + QB_BP - 1) / QB_BP;
  if (ntiles >= (1ll << 31) || (int64_t)QB_BP * N * 2 >= (1ll << 31)) return CESM_EUNSUPPORTED;
  const int nsl = C / 64;
  qkv_bwd_kernel<6><<<(unsigned)(ns * nsl), 512, 0, stream>>>((const bf16*)dy, (const bf16*)x, (const bf16*)wt,
                                                              (bf16*)dx, dw ? slab : nullptr, M, C, (int)ntiles);
  if (dw)
    qkv_bwd_reduce_kernel<<<(unsigned)cdiv((int64_t)N * C, 256), 256, 0, stream>>>(slab, dw, N, C, ns, accumulate);
  return cesm_launch_status();
}

}  // extern "C"
