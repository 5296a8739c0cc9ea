// Weight gradient of the implicit-GEMM convolutions (gfx950, MFMA).
//
//   ws[s][m][tap*ndim + nd] = sum_{p in split s} A[p][m] * B[gather(p, tap)][nd]
//
// A = the per-pixel operand on the reduction grid (n, h, w): dYpre for Conv2d
// (rows = output channels), the input X for ConvTranspose2d (rows = input
// channels).  B = the gathered operand: X under the conv's taps (RDN_G_CONV3:
// 3x3 pad 1 at the same resolution; RDN_G_S2: (2y+dy, 2x+dx) on the 2h x 2w
// grid, which is both Conv2d k2 s2's input and ConvTranspose2d k2 s2's output
// gradient).  The K dimension (pixels) is split over blockIdx.z; a second
// kernel sums the splits in a fixed order (deterministic) and writes the
// reference's OIHW / IOHW layout (aten convolution_backward grad_weight of
// Unet_model.py:26,35-36,48-49,60-61,72-75).
//
// Pixels are staged into LDS as [pixel][channel] rows; MFMA operands need the
// pixel (k) index contiguous per lane, so bf16 fragments come out of LDS with
// the gfx950 transpose read ds_read_b64_tr_b16 and fp32 fragments with one
// ds_read_b32 per lane (v_mfma_f32_16x16x4_f32 takes one k per lane group).
#include "rdn_common.h"

#include <cstdlib>

namespace {

constexpr int NT = 256;
constexpr int KP = 32;  // pixels per stage

template <typename T, int BM, int BN, int WMW, int GATHER>
__global__ __launch_bounds__(NT) void wgrad_kernel(rdn_wgrad_desc d, FastDiv fd_w, FastDiv fd_hw, int pchunk) {
  constexpr int VEC = TypeInfo<T>::VEC;
  constexpr int ES = sizeof(T);
  constexpr int WNW = 4 / WMW;
  constexpr int WTM = BM / WMW, WTN = BN / WNW;
  constexpr int MT = WTM / 16, NTL = WTN / 16;
  constexpr int AG = BM / VEC, BG = BN / VEC;          // 16-B groups per LDS row
  constexpr int A_UNITS = KP * AG, B_UNITS = KP * BG;
  constexpr int A_IT = (A_UNITS + NT - 1) / NT, B_IT = (B_UNITS + NT - 1) / NT;
  constexpr int ROWA = BM * ES + 16, ROWB = BN * ES + 16;
  constexpr int TAPS = GATHER == RDN_G_CONV3 ? 9 : 4;
  static_assert(NT % AG == 0 && NT % BG == 0, "group");

  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * KP * (ROWA + ROWB)];
#define ldsA(b) (lds + (b) * (KP * ROWA))
#define ldsB(b) (lds + 2 * KP * ROWA + (b) * (KP * ROWB))

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WMW, wn = wave / WMW;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int ncol = TAPS * d.ndim;
  const int64_t P = (int64_t)d.n * d.h * d.w;
  const int64_t pbeg = (int64_t)blockIdx.z * pchunk;
  const int64_t pend = pbeg + pchunk < P ? pbeg + pchunk : P;
  const T* __restrict__ A = (const T*)d.a;
  const T* __restrict__ B = (const T*)d.b;

  // fixed channel group per thread
  const int ag = tid % AG, bg = tid % BG;
  const int am = m0 + ag * VEC;
  const bool a_col_ok = am < d.mdim;
  const int bcol = n0 + bg * VEC;
  const bool b_col_ok = bcol < ncol;
  const int btap = b_col_ok ? bcol / d.ndim : 0;
  const int bnd = bcol - btap * d.ndim;
  // channel offsets (channel-blocked operands: rdn_coff), fixed per thread
  const int64_t a_cf = rdn_coff(d.a_c0 + am, d.a_ps, d.a_pl);
  const int64_t b_cf = rdn_coff(d.b_c0 + bnd, d.b_ps, d.b_pl);
  int bdy, bdx;
  if (GATHER == RDN_G_CONV3) { bdy = btap / 3 - 1; bdx = btap % 3 - 1; }
  else { bdy = btap >> 1; bdx = btap & 1; }

  u32x4 ra[A_IT], rb[B_IT];
  auto load_stage = [&](int64_t pb) {
#pragma unroll
    for (int r = 0; r < A_IT; ++r) {
      const int u = tid + r * NT;
      const int64_t p = pb + u / AG;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (u < A_UNITS && a_col_ok && p < pend) v = *(const u32x4*)(A + p * d.a_ps + a_cf);
      ra[r] = v;
    }
#pragma unroll
    for (int r = 0; r < B_IT; ++r) {
      const int u = tid + r * NT;
      const int64_t p = pb + u / BG;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (u < B_UNITS && b_col_ok && p < pend) {
        const uint32_t nimg = fdiv((uint32_t)p, fd_hw);
        const uint32_t rem = (uint32_t)p - nimg * (uint32_t)(d.h * d.w);
        const int y = (int)fdiv(rem, fd_w);
        const int x = (int)rem - y * d.w;
        int ys, xs;
        if (GATHER == RDN_G_CONV3) { ys = y + bdy; xs = x + bdx; }
        else { ys = 2 * y + bdy; xs = 2 * x + bdx; }
        if (ys >= 0 && ys < d.hin && xs >= 0 && xs < d.win)
          v = *(const u32x4*)(B + (((int64_t)nimg * d.hin + ys) * d.win + xs) * d.b_ps + b_cf);
      }
      rb[r] = v;
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int r = 0; r < A_IT; ++r) {
      const int u = tid + r * NT;
      if (u < A_UNITS) *(u32x4*)(ldsA(buf) + (u / AG) * ROWA + ag * 16) = ra[r];
    }
#pragma unroll
    for (int r = 0; r < B_IT; ++r) {
      const int u = tid + r * NT;
      if (u < B_UNITS) *(u32x4*)(ldsB(buf) + (u / BG) * ROWB + bg * 16) = rb[r];
    }
  };

  f32x4 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nst = (int)((pend - pbeg + KP - 1) / KP);
  const int g = lane >> 4, li = lane & 15;
  if (nst > 0) {
    load_stage(pbeg);
    store_stage(0);
  }
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) load_stage(pbeg + (int64_t)(s + 1) * KP);
    if constexpr (ES == 2) {
      // transpose reads: lane 16g+4q+p supplies row (8g+q [+4]) cols (4p..4p+3)
      const int q = li >> 2, pp = li & 3;
      bf16x8 af[MT], bfr[NTL];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const unsigned char* base = ldsA(buf) + (8 * g + q) * ROWA + (wm * WTM + i * 16 + 4 * pp) * 2;
        i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, base));
        i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, base + 4 * ROWA));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < NTL; ++j) {
        const unsigned char* base = ldsB(buf) + (8 * g + q) * ROWB + (wn * WTN + j * 16 + 4 * pp) * 2;
        i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, base));
        i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, base + 4 * ROWB));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < KP / 4; ++e) {
        float af[MT], bfr[NTL];
#pragma unroll
        for (int i = 0; i < MT; ++i)
          af[i] = *(const float*)(ldsA(buf) + (4 * e + g) * ROWA + (wm * WTM + i * 16 + li) * 4);
#pragma unroll
        for (int j = 0; j < NTL; ++j)
          bfr[j] = *(const float*)(ldsB(buf) + (4 * e + g) * ROWB + (wn * WTN + j * 16 + li) * 4);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NTL; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (s + 1 < nst) store_stage(buf ^ 1);
    __syncthreads();
  }

#undef ldsA
#undef ldsB
  float* __restrict__ ws = d.ws + (int64_t)blockIdx.z * d.mdim * ncol;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) {
      const int col = n0 + wn * WTN + j * 16 + li;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * WTM + i * 16 + g * 4 + e;
        if (m < d.mdim && col < ncol) ws[(int64_t)m * ncol + col] = acc[i][j][e];
      }
    }
}

// Split reduction: block = CPB consecutive workspace columns x SL split lanes
// (consecutive threads -> consecutive columns: coalesced slab reads); each
// thread sums splits sl, sl+SL, ... and the SL partials are added in a fixed
// order through LDS (deterministic).  The result goes to the reference layout
// [m][nd][tap] (OIHW / IOHW).
// one block of a reduction: slab block `bx` (part == false) or partial block `bx`
// (part == true: one per (channel, dalpha|dbias), fixed order)
__device__ __forceinline__ void wgrad_reduce_block(const float* __restrict__ ws, int splits, int mdim, int ndim,
                                                   int ndim_real, int taps, float* __restrict__ grad, int accumulate,
                                                   int sl_count, const float* __restrict__ part, int part_splits,
                                                   float* __restrict__ dalpha, float* __restrict__ dbias, int gstride,
                                                   int gci0, int bx, bool is_part) {
  if (is_part) {  // fused-PReLU partials
    if (bx >= 2 * mdim) return;
    const int which = bx / mdim, m = bx - which * mdim;
    float s = 0.f;
    for (int z = threadIdx.x; z < part_splits; z += 256) s += part[((int64_t)z * 2 + which) * mdim + m];
    __shared__ float red1[256];
    red1[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (threadIdx.x < o) red1[threadIdx.x] += red1[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      float* dst = which ? dbias : dalpha;
      if (dst) dst[m] += red1[0];
    }
    return;
  }
  // 4 consecutive columns per thread (16-B loads), sl_count split lanes per
  // column quad, lanes combined in LDS in a fixed order (deterministic)
  const int qpb = 256 / sl_count;                 // column quads per block
  const int cq = threadIdx.x % qpb, sl = threadIdx.x / qpb;
  const int ncol = taps * ndim;
  const int64_t total = (int64_t)mdim * ncol;     // multiple of 4 (ndim % 8 == 0)
  const int64_t o = ((int64_t)bx * qpb + cq) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (o < total) {
    const float* p = ws + o;
    int z = sl;
    for (; z + 3 * sl_count < splits; z += 4 * sl_count) {
      const f32x4 a0 = *(const f32x4*)(p + (int64_t)z * total);
      const f32x4 a1 = *(const f32x4*)(p + (int64_t)(z + sl_count) * total);
      const f32x4 a2 = *(const f32x4*)(p + (int64_t)(z + 2 * sl_count) * total);
      const f32x4 a3 = *(const f32x4*)(p + (int64_t)(z + 3 * sl_count) * total);
      s += (a0 + a1) + (a2 + a3);
    }
    for (; z < splits; z += sl_count) s += *(const f32x4*)(p + (int64_t)z * total);
  }
  __shared__ f32x4 red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (sl == 0 && o < total) {
    for (int q = 1; q < sl_count; ++q) s += red[q * qpb + cq];
    const int m = (int)(o / ncol);
    const int col0 = (int)(o - (int64_t)m * ncol);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = col0 + e;
      const int tap = col / ndim, nd = col - tap * ndim;
      if (nd < ndim_real) {
        const int64_t dst = ((int64_t)m * gstride + gci0 + nd) * taps + tap;
        grad[dst] = accumulate ? grad[dst] + s[e] : s[e];
      }
    }
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, int splits, int mdim, int ndim,
                                                           int ndim_real, int taps, float* __restrict__ grad,
                                                           int accumulate, int sl_count, const float* __restrict__ part,
                                                           int part_splits, float* __restrict__ dalpha,
                                                           float* __restrict__ dbias, int gstride, int gci0) {
  wgrad_reduce_block(ws, splits, mdim, ndim, ndim_real, taps, grad, accumulate, sl_count, part, part_splits, dalpha,
                     dbias, gstride, gci0, blockIdx.x, blockIdx.y == 1);
}

// Several reductions in ONE launch (round 4): the fused dgrad+wgrad layers' reduces
// run on the compute stream, one small latency-bound launch per layer (40 per B16
// step, ~7 us each against ~2-3 us of slab bytes); consecutive ones go together.
// Job j owns blocks [beg[j], beg[j+1]): its slab blocks, then its partial blocks.
// Same per-block work and summation order as the single launches (bit-identical).
struct ReduceBatch {
  rdn_reduce_job job[RDN_REDUCE_BATCH_MAX];
  int32_t beg[RDN_REDUCE_BATCH_MAX + 1];
  int32_t n;
};

__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(ReduceBatch b) {
  int j = 0;
  while (j + 1 < b.n && (int)blockIdx.x >= b.beg[j + 1]) ++j;
  const rdn_reduce_job& q = b.job[j];
  const int bx = (int)blockIdx.x - b.beg[j];
  const bool is_part = bx >= q.blocks;
  wgrad_reduce_block(q.ws, q.splits, q.mdim, q.ndim, q.ndim_real, q.taps, q.grad, q.accumulate, q.sl, q.part,
                     q.part_splits > 0 ? q.part_splits : q.splits, q.dalpha, q.dbias, q.gstride, q.gci0,
                     is_part ? bx - q.blocks : bx, is_part);
}

struct Cfg { int bm, bn; };
static Cfg pick(const rdn_wgrad_desc* d) {
  const int taps = d->gather == RDN_G_CONV3 ? 9 : 4;
  Cfg c;
  c.bm = d->mdim <= 16 ? 16 : d->mdim <= 32 ? 32 : 64;
  c.bn = taps * d->ndim <= 64 ? 64 : 128;
  return c;
}

static int auto_splits(const rdn_wgrad_desc* d) {
  if (d->splits > 0) return d->splits;
  const Cfg c = pick(d);
  const int taps = d->gather == RDN_G_CONV3 ? 9 : 4;
  const int64_t tiles = (int64_t)((d->mdim + c.bm - 1) / c.bm) * ((taps * d->ndim + c.bn - 1) / c.bn);
  const int64_t P = (int64_t)d->n * d->h * d->w;
  // ~2 blocks per CU (round 4, interleaved: 512 1771 / 1957, 256 1765 / 1939, 128 1767 /
  // 1941 img/s B16 / B32, profiles/r04_v31_wg2_blocks_ab.txt; RDN_WG2_BLOCKS for A/B)
  static const int64_t target = [] {
    const char* e = getenv("RDN_WG2_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return (int64_t)(v > 0 ? v : 512);
  }();
  int64_t s = (target + tiles - 1) / tiles;
  const int64_t maxs = (P + 1023) / 1024;                 // >= 1024 pixels per split
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  return (int)s;
}

template <typename T, int BM, int BN, int WMW>
static int launch_g(const rdn_wgrad_desc* d, hipStream_t st) {
  const int taps = d->gather == RDN_G_CONV3 ? 9 : 4;
  const int splits = auto_splits(d);
  const int64_t P = (int64_t)d->n * d->h * d->w;
  int64_t pchunk = (P + splits - 1) / splits;
  pchunk = (pchunk + KP - 1) / KP * KP;
  dim3 grid((d->mdim + BM - 1) / BM, (taps * d->ndim + BN - 1) / BN, splits);
  FastDiv fw = make_fastdiv((uint32_t)d->w), fhw = make_fastdiv((uint32_t)(d->h * d->w));
  RDN_PROBE("wgrad_kernel<%s,%d,%d,%d,%d>", rdn_tname<T>(), BM, BN, WMW, d->gather);
  if (d->gather == RDN_G_CONV3)
    wgrad_kernel<T, BM, BN, WMW, RDN_G_CONV3><<<grid, NT, 0, st>>>(*d, fw, fhw, (int)pchunk);
  else
    wgrad_kernel<T, BM, BN, WMW, RDN_G_S2><<<grid, NT, 0, st>>>(*d, fw, fhw, (int)pchunk);
  return rdn_check_launch("rdn_conv_wgrad");
}

template <typename T>
static int launch_t(const rdn_wgrad_desc* d, hipStream_t st) {
  const Cfg c = pick(d);
  if (c.bm == 16) return c.bn == 64 ? launch_g<T, 16, 64, 1>(d, st) : launch_g<T, 16, 128, 1>(d, st);
  if (c.bm == 32) return c.bn == 64 ? launch_g<T, 32, 64, 2>(d, st) : launch_g<T, 32, 128, 2>(d, st);
  return c.bn == 64 ? launch_g<T, 64, 64, 2>(d, st) : launch_g<T, 64, 128, 2>(d, st);
}

}  // namespace

extern "C" int rdn_wgrad_splits(const rdn_wgrad_desc* d) {
  if (!d) return RDN_E_ARG;
  return d->gather == RDN_G_CONV3 ? rdn_wgrad3_splits(d) : auto_splits(d);
}

extern "C" int rdn_wgrad_chunks(const rdn_wgrad_desc* d) {
  if (!d) return RDN_E_ARG;
  return d->gather == RDN_G_CONV3 ? rdn_wgrad3_chunks(d) : 1;
}

extern "C" int64_t rdn_wgrad_workspace_size(const rdn_wgrad_desc* d) {
  if (!d) return RDN_E_ARG;
  const int taps = d->gather == RDN_G_CONV3 ? 9 : 4;
  return (int64_t)rdn_wgrad_splits(d) * d->mdim * taps * d->ndim * (int64_t)sizeof(float);
}

extern "C" int rdn_conv_wgrad(const rdn_wgrad_desc* d, void* stream) {
  if (!d || !d->a || !d->b || !d->ws) { rdn_set_error("rdn_conv_wgrad: null pointer"); return RDN_E_ARG; }
  if (d->dtype != RDN_F32 && d->dtype != RDN_BF16) { rdn_set_error("rdn_conv_wgrad: bad dtype"); return RDN_E_ARG; }
  if (d->gather != RDN_G_CONV3 && d->gather != RDN_G_S2) { rdn_set_error("rdn_conv_wgrad: bad gather"); return RDN_E_ARG; }
  const int vec = d->dtype == RDN_BF16 ? 8 : 4;
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->mdim <= 0 || d->ndim <= 0) { rdn_set_error("rdn_conv_wgrad: empty shape"); return RDN_E_SHAPE; }
  if (d->ndim % 8 || d->a_ps % vec || d->a_c0 % vec || d->b_ps % vec || d->b_c0 % vec ||
      ((uintptr_t)d->a & 15) || ((uintptr_t)d->b & 15)) {
    rdn_set_error("rdn_conv_wgrad: alignment (ndim=%d a_ps=%lld a_c0=%d b_ps=%lld b_c0=%d)", d->ndim,
                  (long long)d->a_ps, d->a_c0, (long long)d->b_ps, d->b_c0);
    return RDN_E_SHAPE;
  }
  if ((d->a_pl && rdn_coff(d->a_c0 + d->mdim - 1, d->a_ps, d->a_pl) >= (1ll << 31)) ||
      (d->b_pl && rdn_coff(d->b_c0 + d->ndim - 1, d->b_ps, d->b_pl) >= (1ll << 31))) {
    rdn_set_error("rdn_conv_wgrad: channel-blocked operand offsets must stay below 2^31 elements");
    return RDN_E_SHAPE;
  }
  if (d->gather == RDN_G_S2 ? (d->hin != 2 * d->h || d->win != 2 * d->w) : (d->hin != d->h || d->win != d->w)) {
    rdn_set_error("rdn_conv_wgrad: grid mismatch"); return RDN_E_SHAPE;
  }
  if ((int64_t)d->n * d->h * d->w >= (1ll << 31)) { rdn_set_error("rdn_conv_wgrad: too many pixels"); return RDN_E_SHAPE; }
  hipStream_t st = (hipStream_t)stream;
  if (d->gather == RDN_G_CONV3) return rdn_wgrad3_launch(d, st);  // LDS-halo kernel (wgrad3_halo.hip)
  return d->dtype == RDN_BF16 ? launch_t<bf16>(d, st) : launch_t<float>(d, st);
}

// split lanes per column quad: only as many as it takes to give the launch ~64k
// threads (one per lane of every SIMD); each lane then streams its splits with
// four loads in flight.  (Lanes for every split up to 16 -- the previous rule --
// left the wide level-2/3 reductions at one or two loads per thread: 0.7 TB/s.)
static int reduce_lanes(int64_t total, int splits) {
  const int64_t quads = total / 4;
  int sl = 1;
  while (sl < 16 && sl < splits && quads * sl < 65536) sl <<= 1;
  return sl;
}

static int wgrad_reduce_impl(const float* ws, int32_t splits, int32_t mdim, int32_t ndim, int32_t ndim_real,
                             int32_t taps, float* grad, int32_t gstride, int32_t gci0, int32_t accumulate,
                             const float* part, int32_t part_splits, float* dalpha, float* dbias, void* stream) {
  if (!ws || !grad || splits <= 0 || mdim <= 0 || ndim <= 0 || ndim_real <= 0 || ndim_real > ndim || taps <= 0 ||
      gci0 < 0 || gci0 + ndim_real > gstride) {
    rdn_set_error("rdn_wgrad_reduce: bad arguments"); return RDN_E_ARG;
  }
  const int64_t total = (int64_t)mdim * ndim * taps;
  if (ndim % 4 || ((uintptr_t)ws & 15)) { rdn_set_error("rdn_wgrad_reduce: ndim %% 4 / alignment"); return RDN_E_ARG; }
  const int sl = reduce_lanes(total, splits);
  const int qpb = 256 / sl;
  int64_t blocks = (total / 4 + qpb - 1) / qpb;
  if (part && blocks < 2 * mdim) blocks = 2 * mdim;
  if (blocks > 0x7fffffff) { rdn_set_error("rdn_wgrad_reduce: too large"); return RDN_E_SHAPE; }
  dim3 grid((unsigned)blocks, part ? 2 : 1);
  wgrad_reduce_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(ws, splits, mdim, ndim, ndim_real, taps, grad, accumulate,
                                                            sl, part, part_splits > 0 ? part_splits : splits, dalpha,
                                                            dbias, gstride, gci0);
  return rdn_check_launch("rdn_wgrad_reduce");
}

extern "C" int rdn_wgrad_reduce(const float* ws, int32_t splits, int32_t mdim, int32_t ndim, int32_t ndim_real,
                                int32_t taps, float* grad, int32_t accumulate, const float* part, int32_t part_splits,
                                float* dalpha, float* dbias, void* stream) {
  return wgrad_reduce_impl(ws, splits, mdim, ndim, ndim_real, taps, grad, ndim_real, 0, accumulate, part, part_splits,
                           dalpha, dbias, stream);
}

extern "C" int rdn_wgrad_reduce_cols(const float* ws, int32_t splits, int32_t mdim, int32_t ndim, int32_t taps,
                                     float* grad, int32_t grad_ci_total, int32_t grad_ci0, int32_t accumulate,
                                     const float* part, int32_t part_splits, float* dalpha, float* dbias,
                                     void* stream) {
  return wgrad_reduce_impl(ws, splits, mdim, ndim, ndim, taps, grad, grad_ci_total, grad_ci0, accumulate, part,
                           part_splits, dalpha, dbias, stream);
}

// Up to RDN_REDUCE_BATCH_MAX reductions (each as rdn_wgrad_reduce_cols would run it:
// ws, splits, mdim, ndim, ndim_real, taps, grad + gstride / gci0, accumulate, the
// fused-PReLU partials) in one launch; sl / blocks are filled in here.
extern "C" int rdn_wgrad_reduce_batch(const rdn_reduce_job* jobs, int32_t n, void* stream) {
  if (!jobs || n <= 0 || n > RDN_REDUCE_BATCH_MAX) { rdn_set_error("rdn_wgrad_reduce_batch: 1..%d jobs", RDN_REDUCE_BATCH_MAX); return RDN_E_ARG; }
  ReduceBatch b{};
  b.n = n;
  int64_t acc = 0;
  for (int j = 0; j < n; ++j) {
    rdn_reduce_job q = jobs[j];
    if (!q.ws || !q.grad || q.splits <= 0 || q.mdim <= 0 || q.ndim <= 0 || q.ndim_real <= 0 || q.ndim_real > q.ndim ||
        q.taps <= 0 || q.gci0 < 0 || q.gci0 + q.ndim_real > q.gstride || q.ndim % 4 || ((uintptr_t)q.ws & 15)) {
      rdn_set_error("rdn_wgrad_reduce_batch: job %d: bad arguments", j);
      return RDN_E_ARG;
    }
    const int64_t total = (int64_t)q.mdim * q.ndim * q.taps;
    q.sl = reduce_lanes(total, q.splits);
    const int qpb = 256 / q.sl;
    q.blocks = (int32_t)((total / 4 + qpb - 1) / qpb);
    q.pblocks = q.part ? 2 * q.mdim : 0;
    b.job[j] = q;
    b.beg[j] = (int32_t)acc;
    acc += (int64_t)q.blocks + q.pblocks;
  }
  if (acc > 0x7fffffff) { rdn_set_error("rdn_wgrad_reduce_batch: too large"); return RDN_E_SHAPE; }
  b.beg[n] = (int32_t)acc;
  wgrad_reduce_batch_kernel<<<(unsigned)acc, 256, 0, (hipStream_t)stream>>>(b);
  return rdn_check_launch("rdn_wgrad_reduce_batch");
}
