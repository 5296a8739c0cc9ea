// Weight gradient of the 3x3 / pad 1 convolutions with an LDS input halo
// (gfx950, MFMA):
//
//   ws[split][co][tap*ndim + ci] = sum_p dYpre[p][co] * X[p + tap][ci]
//
// Block = (BM output channels) x (one CK-channel chunk of the input) x a range
// of 8 x 16 pixel tiles.  Per tile the dYpre tile [128 px][BM] and the input
// halo [(8+2) x (16+2) px][CK] are staged into LDS ONCE and feed all 9 taps
// (the generic path re-gathers the input once per tap), giving BM x 9*CK
// accumulators per block with K = 128 pixels per tile.
//
// MFMA operands need the pixel (k) index along each lane's 8 elements, so
// bf16 fragments come out of LDS with ds_read_b64_tr_b16 (each 16-lane group
// reads 4 pixel rows x 16 channels and gets it transposed).  Lane group g
// takes pixels {4g..4g+3} then {16+4g..16+4g+3} of a 32-pixel k-step, so the
// 8 rows a half-wave touches are consecutive: with the padded row strides
// below every transpose read is bank-conflict free.  fp32 takes one pixel per
// lane group (v_mfma_f32_16x16x4_f32) with plain ds_read_b32.
//
// The dYpre tile of image pixels outside the image is zero, so partial tiles
// contribute nothing.  Splits are summed by rdn_wgrad_reduce (fixed order).
#include "rdn_common.h"

#include <cstdlib>

namespace {

constexpr int NT = 256;
constexpr int TH = 8, TW = 16, TP = TH * TW;
constexpr int HP = (TH + 2) * (TW + 2);

// conflict-free row strides for ds_read_b64_tr_b16 with the interleaved
// k order (see header): data bytes -> stride
constexpr int tr_stride(int bytes) {
  return bytes <= 32 ? bytes : bytes == 64 ? 96 : bytes == 96 ? 96 : bytes == 128 ? 160 : bytes == 160 ? 160
       : bytes == 192 ? 224 : bytes + 32;
}
// fp32 (ds_read_b32, rows g and g+1 in one half-wave): stride = 64 (mod 128) bytes
constexpr int f32_stride(int bytes) { return bytes % 128 <= 64 ? bytes - bytes % 128 + 64 : bytes - bytes % 128 + 192; }

template <typename T, int BM, int CK, bool GATE>
__global__ __launch_bounds__(NT, 2) void wgrad3_halo_kernel(rdn_wgrad_desc d, int tiles_x, int tiles_y, int ntiles,
                                                            int tiles_per_block) {
  constexpr int ES = sizeof(T);
  constexpr int VEC = TypeInfo<T>::VEC;
  constexpr int NCOL = 9 * CK;
  constexpr int NT_ALL = (NCOL + 15) / 16;
  constexpr int NTW = (NT_ALL + 3) / 4;     // n-tiles per wave
  constexpr int MT = BM / 16;
  constexpr int DROW = ES == 2 ? tr_stride(BM * ES) : f32_stride(BM * ES);
  constexpr int HROW = ES == 2 ? tr_stride(CK * ES) : f32_stride(CK * ES);
  constexpr int D_UNITS = TP * (BM / VEC), H_UNITS = HP * (CK / VEC);
  constexpr int D_IT = (D_UNITS + NT - 1) / NT, H_IT = (H_UNITS + NT - 1) / NT;
  constexpr int D_BYTES = TP * DROW;
  constexpr int MAIN_BYTES = D_BYTES + HP * HROW;
  constexpr int RED_BYTES = GATE ? 2 * NT * VEC * 4 : 0;   // dalpha/dbias partial reduction
  __shared__ __attribute__((aligned(16))) unsigned char lds[MAIN_BYTES > RED_BYTES ? MAIN_BYTES : RED_BYTES];
  unsigned char* const dyl = lds;
  unsigned char* const hal = lds + D_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * BM;
  const int c0 = blockIdx.y * CK;
  const int t_beg = blockIdx.z * tiles_per_block;
  const int t_end = min(t_beg + tiles_per_block, ntiles);
  const T* __restrict__ A = (const T*)d.a;
  const T* __restrict__ Bx = (const T*)d.b;
  const int H = d.h, W = d.w;

  u32x4 dreg[D_IT], hreg[H_IT];
  // PReLU-backward gate on A (dY -> dYpre) + dalpha / dbias partials
  static_assert(NT % (BM / VEC) == 0, "fixed channel group per thread");
  u32x4 greg[GATE ? D_IT : 1];
  const T* __restrict__ G = (const T*)d.a_gate;
  const int acg = tid % (BM / VEC);           // this thread's A channel group
  float galpha[GATE ? VEC : 1], sa[GATE ? VEC : 1], sb[GATE ? VEC : 1];
  const bool do_part = GATE && d.part != nullptr && blockIdx.y == 0;
  if constexpr (GATE) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const int m = m0 + acg * VEC + q;
      galpha[q] = m < d.mdim ? d.a_gate_alpha[m] : 0.f;
      sa[q] = 0.f;
      sb[q] = 0.f;
    }
  }
  // channel offsets of this thread's A and B units: the unit's channel group is the
  // same in every iteration (NT is a multiple of both unit counts per pixel), so
  // the channel-blocked decode (rdn_coff) runs once
  const int a_cf = rdn_coff32(d.a_c0 + m0 + acg * VEC, (int)d.a_ps, (int)d.a_pl);
  const int g_cf = GATE ? rdn_coff32(m0 + acg * VEC, (int)d.a_gate_ps, (int)d.a_gate_pl) : 0;
  static_assert(NT % (CK / VEC) == 0, "fixed B channel group per thread");
  const int b_cf = rdn_coff32(d.b_c0 + c0 + (tid % (CK / VEC)) * VEC, (int)d.b_ps, (int)d.b_pl);
  auto load_tile = [&](int t) {
    const int tx = t % tiles_x, r1 = t / tiles_x;
    const int ty = r1 % tiles_y, nimg = r1 / tiles_y;
    const int y0 = ty * TH, x0 = tx * TW;
#pragma unroll
    for (int it = 0; it < D_IT; ++it) {
      const int u = tid + it * NT;
      u32x4 v = {0u, 0u, 0u, 0u}, gv = {0u, 0u, 0u, 0u};
      if (u < D_UNITS) {
        const int p = u / (BM / VEC), cu = u - p * (BM / VEC);
        const int yy = y0 + p / TW, xx = x0 + p % TW;
        const int m = m0 + cu * VEC;
        if (yy < H && xx < W && m < d.mdim) {
          const int64_t pix = ((int64_t)nimg * H + yy) * W + xx;
          v = *(const u32x4*)(A + pix * d.a_ps + a_cf);
          if constexpr (GATE) gv = *(const u32x4*)(G + pix * d.a_gate_ps + g_cf);
        }
      }
      dreg[it] = v;
      if constexpr (GATE) greg[it] = gv;
    }
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      const int u = tid + it * NT;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (u < H_UNITS) {
        const int hp = u / (CK / VEC), cu = u - hp * (CK / VEC);
        const int hy = hp / (TW + 2), hx = hp - hy * (TW + 2);
        const int yy = y0 + hy - 1, xx = x0 + hx - 1;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
          v = *(const u32x4*)(Bx + (((int64_t)nimg * H + yy) * W + xx) * d.b_ps + b_cf);
      }
      hreg[it] = v;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int it = 0; it < D_IT; ++it) {
      const int u = tid + it * NT;
      if (u < D_UNITS) {
        const int p = u / (BM / VEC), cu = u - p * (BM / VEC);
        u32x4 v = dreg[it];
        if constexpr (GATE) {
          float dy[VEC], pr[VEC];
          Unit16<T>::unpack(v, dy);
          Unit16<T>::unpack(greg[it], pr);
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            const bool pos = pr[q] > 0.f;
            if (!pos) sa[q] += pr[q] * dy[q];
            dy[q] = pos ? dy[q] : galpha[q] * dy[q];
          }
          v = Unit16<T>::pack(dy);
          if (do_part) {  // dbias sums dYpre before its rounding to T, as rdn_prelu_bwd does
#pragma unroll
            for (int q = 0; q < VEC; ++q) sb[q] += dy[q];
          }
        }
        *(u32x4*)(dyl + p * DROW + cu * 16) = v;
      }
    }
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      const int u = tid + it * NT;
      if (u < H_UNITS) {
        const int hp = u / (CK / VEC), cu = u - hp * (CK / VEC);
        *(u32x4*)(hal + hp * HROW + cu * 16) = hreg[it];
      }
    }
  };

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per n-tile of this wave: tap offset and channel of this lane's column(s)
  int col_tap[NTW], col_ci[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wave + 4 * j;
    // bf16: lane supplies columns (4p .. 4p+3) of the tile; fp32: column li
    const int c = nt * 16 + (ES == 2 ? 4 * (li & 3) : li);
    const int cc = (nt < NT_ALL && c < NCOL) ? c : 0;
    col_tap[j] = cc / CK;
    col_ci[j] = cc - (cc / CK) * CK;
  }

  if (t_beg < t_end) {
    load_tile(t_beg);
    store_tile();
  }
  __syncthreads();
  for (int t = t_beg; t < t_end; ++t) {
    if (t + 1 < t_end) load_tile(t + 1);
    if constexpr (ES == 2) {
      const int q = li >> 2, pp = li & 3;
#pragma unroll
      for (int ks = 0; ks < TP / 32; ++ks) {
        // k slots of group g: pixels ks*32 + {4g+q} and ks*32 + 16 + {4g+q}
        const int pa = ks * 32 + 4 * g + q, pb = pa + 16;
        bf16x8 af[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, dyl + pa * DROW + (i * 16 + 4 * pp) * 2));
          const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, dyl + pb * DROW + (i * 16 + 4 * pp) * 2));
          af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
        const int pya = pa >> 4, pxa = pa & 15, pyb = pb >> 4, pxb = pb & 15;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          if (wave + 4 * j >= NT_ALL) continue;
          const int tp = col_tap[j], ky = tp / 3, kx = tp - 3 * ky;
          const unsigned char* ba = hal + ((pya + ky) * (TW + 2) + pxa + kx) * HROW + col_ci[j] * 2;
          const unsigned char* bb = hal + ((pyb + ky) * (TW + 2) + pxb + kx) * HROW + col_ci[j] * 2;
          const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, ba));
          const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, bb));
          const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int i = 0; i < MT; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
        }
      }
    } else {
#pragma unroll 4
      for (int e = 0; e < TP / 4; ++e) {
        const int p = 4 * e + g;
        const int py = p >> 4, px = p & 15;
        float af[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i] = *(const float*)(dyl + p * DROW + (i * 16 + li) * 4);
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          if (wave + 4 * j >= NT_ALL) continue;
          const int tp = col_tap[j], ky = tp / 3, kx = tp - 3 * ky;
          const float b = *(const float*)(hal + ((py + ky) * (TW + 2) + px + kx) * HROW + col_ci[j] * 4);
#pragma unroll
          for (int i = 0; i < MT; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], b, acc[i][j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
    if (t + 1 < t_end) {
      store_tile();
      __syncthreads();
    }
  }

  if constexpr (GATE) {
    if (d.part != nullptr && blockIdx.y == 0) {
      // per-block channel partials -> part[split][0|1][m] (LDS reduce, fixed order)
      float* red = (float*)lds;  // reuse: the tile loop ended with a barrier
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        red[tid * VEC + q] = sa[q];
        red[NT * VEC + tid * VEC + q] = sb[q];
      }
      __syncthreads();
      constexpr int GPB = BM / VEC;
      if (tid < BM) {
        const int cg = tid / VEC, q = tid % VEC;
        float a = 0.f, b = 0.f;
        for (int k = 0; k < NT / GPB; ++k) {
          a += red[(k * GPB + cg) * VEC + q];
          b += red[NT * VEC + (k * GPB + cg) * VEC + q];
        }
        const int m = m0 + tid;
        if (m < d.mdim) {
          d.part[((int64_t)blockIdx.z * 2 + 0) * d.mdim + m] = a;
          d.part[((int64_t)blockIdx.z * 2 + 1) * d.mdim + m] = b;
        }
      }
    }
  }
  // D[m][n]: row = g*4 + e (output channel), col = li (tile column)
  const int ncol_all = 9 * d.ndim;
  float* __restrict__ ws = d.ws + (int64_t)blockIdx.z * d.mdim * ncol_all;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wave + 4 * j;
    const int c = nt * 16 + li;
    if (nt >= NT_ALL || c >= NCOL) continue;
    const int tp = c / CK, ci = c - tp * CK;
    const int col = tp * d.ndim + c0 + ci;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + i * 16 + g * 4 + e;
        if (m < d.mdim) ws[(int64_t)m * ncol_all + col] = acc[i][j][e];
      }
  }
}

// bf16 variant with wide channel groups (CK up to 96: whole level-0 pixel rows,
// so dY and X are each read once per launch in full rows) and no per-tile
// index math in the k loop: every LDS operand address is a per-thread base
// fixed for the launch plus an immediate, and the tile loaders add one
// precomputed per-unit offset to a per-tile base.
template <int BM, int CK, bool GATE>
__global__ __launch_bounds__(NT, (BM * CK > 2560 ? 1 : 2)) void wgrad3_rows_kernel(rdn_wgrad_desc d, int tiles_x, int tiles_y, int ntiles,
                                                            int tiles_per_block) {
  constexpr int VEC = 8;
  constexpr int NCOL = 9 * CK;
  constexpr int NT_ALL = (NCOL + 15) / 16;
  constexpr int NTW = (NT_ALL + 3) / 4;     // n-tiles per wave (n-tile = wave + 4 j)
  constexpr int MT = BM / 16;
  constexpr int DROW = tr_stride(BM * 2);
  constexpr int HROW = tr_stride(CK * 2);
  constexpr int DU = BM / VEC, HU = CK / VEC;   // 16-B units per pixel row
  constexpr int D_UNITS = TP * DU, H_UNITS = HP * HU;
  constexpr int D_IT = (D_UNITS + NT - 1) / NT, H_IT = (H_UNITS + NT - 1) / NT;
  constexpr int D_BYTES = TP * DROW;
  constexpr int MAIN_BYTES = D_BYTES + HP * HROW;
  constexpr int RED_BYTES = GATE ? 2 * NT * VEC * 4 : 0;
  static_assert(NT % DU == 0, "fixed dY channel group per thread");
  __shared__ __attribute__((aligned(16))) unsigned char lds[MAIN_BYTES > RED_BYTES ? MAIN_BYTES : RED_BYTES];
  unsigned char* const dyl = lds;
  unsigned char* const hal = lds + D_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  // 1-D grid, logical (m-tile, chunk, split) with the m-tile fastest, remapped so
  // that consecutive logical blocks share an XCD (xcd_remap): the chunks and
  // m-tiles of one pixel range then read its dY / X tiles through ONE L2.  With
  // the plain order they spread over all 8 XCDs: level-2/3 wgrad HBM traffic
  // 195 MB -> 74 MB per launch (PMC, 4.0x -> 1.5x the algorithmic bytes) at the
  // same step time beside the dgrad chain (isolated the plain order was faster)
  const int mtiles = (d.mdim + BM - 1) / BM, nchunks = d.ndim / CK;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int bx = lb % mtiles, by = (lb / mtiles) % nchunks, bz = lb / (mtiles * nchunks);
  const int m0 = bx * BM;
  const int c0 = by * CK;
  const int t_beg = bz * tiles_per_block;
  const int t_end = min(t_beg + tiles_per_block, ntiles);
  const int H = d.h, W = d.w;
  const bf16* __restrict__ A = (const bf16*)d.a;
  const bf16* __restrict__ Bx = (const bf16*)d.b;
  const bf16* __restrict__ G = (const bf16*)d.a_gate;

  // ---- per-thread unit geometry (tile-invariant)
  const int acg = tid % DU;                     // this thread's dY channel group
  const bool m_ok = m0 + acg * VEC < d.mdim;
  const int a_cf = rdn_coff32(d.a_c0 + m0 + acg * VEC, (int)d.a_ps, (int)d.a_pl);   // channel-blocked decode, once
  const int g_cf = GATE ? rdn_coff32(m0 + acg * VEC, (int)d.a_gate_ps, (int)d.a_gate_pl) : 0;
  int drel[D_IT], grel[GATE ? D_IT : 1];
#pragma unroll
  for (int it = 0; it < D_IT; ++it) {
    const int p = (tid + it * NT) / DU;
    drel[it] = ((p / TW) * W + p % TW) * (int)d.a_ps + a_cf;
    if constexpr (GATE) grel[it] = ((p / TW) * W + p % TW) * (int)d.a_gate_ps + g_cf;
  }
  // pixel of dY unit `it` and its LDS offset (constant divisors: no tables)
  auto dpix = [&](int it) { return (tid + it * NT) / DU; };
  auto dlds = [&](int it) { return dpix(it) * DROW + acg * 16; };
  constexpr bool HLIN = HROW == HU * 16;        // unpadded halo rows: LDS offset = unit * 16
  int hrel[H_IT], hlds[HLIN ? 1 : H_IT];
#pragma unroll
  for (int it = 0; it < H_IT; ++it) {
    const int u = tid + it * NT;
    const int hp = u / HU, cu = u - hp * HU;
    const int hy = hp / (TW + 2), hx = hp - hy * (TW + 2);
    hrel[it] = (hy * W + hx) * (int)d.b_ps + rdn_coff32(d.b_c0 + c0 + cu * VEC, (int)d.b_ps, (int)d.b_pl);
    if constexpr (!HLIN) hlds[it] = hp * HROW + cu * 16;
  }

  float galpha[GATE ? VEC : 1], sa[GATE ? VEC : 1], sb[GATE ? VEC : 1];
  const bool do_part = GATE && d.part != nullptr && by == 0;
  if constexpr (GATE) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const int m = m0 + acg * VEC + q;
      galpha[q] = m < d.mdim ? d.a_gate_alpha[m] : 0.f;
      sa[q] = 0.f;
      sb[q] = 0.f;
    }
  }

  constexpr int GD = GATE ? D_IT : 1;
  auto load_tile = [&](int t, u32x4 (&dreg)[D_IT], u32x4 (&greg)[GD], u32x4 (&hreg)[H_IT]) {
    const int tx = t % tiles_x, r1 = t / tiles_x;
    const int ty = r1 % tiles_y, nimg = r1 / tiles_y;
    const int y0 = ty * TH, x0 = tx * TW;
    const int64_t pix0 = ((int64_t)nimg * H + y0) * W + x0;
    const bool full = y0 + TH <= H && x0 + TW <= W;
    const bf16* const ab = A + pix0 * d.a_ps;
    const bf16* const gb = GATE ? G + pix0 * d.a_gate_ps : nullptr;
#pragma unroll
    for (int it = 0; it < D_IT; ++it) {
      const int p = dpix(it);
      bool ok = m_ok && ((it + 1 < D_IT) || tid + it * NT < D_UNITS);
      if (!full) ok = ok && y0 + p / TW < H && x0 + p % TW < W;
      u32x4 v = {0u, 0u, 0u, 0u}, gv = {0u, 0u, 0u, 0u};
      if (ok) {
        v = *(const u32x4*)(ab + drel[it]);
        if constexpr (GATE) gv = *(const u32x4*)(gb + grel[it]);
      }
      dreg[it] = v;
      if constexpr (GATE) greg[it] = gv;
    }
    const bf16* const hb = Bx + (pix0 - W - 1) * d.b_ps;   // halo pixel (0, 0) = image (y0 - 1, x0 - 1)
    const bool interior = y0 >= 1 && y0 + TH + 1 <= H && x0 >= 1 && x0 + TW + 1 <= W;
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      const int u = tid + it * NT;
      bool ok = (it + 1 < H_IT) || u < H_UNITS;
      if (!interior) {
        const int hp = u / HU;
        const int hy = hp / (TW + 2), hx = hp - hy * (TW + 2);
        ok = ok && (unsigned)(y0 - 1 + hy) < (unsigned)H && (unsigned)(x0 - 1 + hx) < (unsigned)W;
      }
      u32x4 v = {0u, 0u, 0u, 0u};
      if (ok) v = *(const u32x4*)(hb + hrel[it]);
      hreg[it] = v;
    }
  };
  auto store_tile = [&](const u32x4 (&dreg)[D_IT], const u32x4 (&greg)[GD], const u32x4 (&hreg)[H_IT]) {
#pragma unroll
    for (int it = 0; it < D_IT; ++it) {
      if (it + 1 == D_IT && tid + it * NT >= D_UNITS) continue;
      u32x4 v = dreg[it];
      if constexpr (GATE) {
        float dy[VEC], pr[VEC];
        Unit16<bf16>::unpack(v, dy);
        Unit16<bf16>::unpack(greg[it], pr);
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          const bool pos = pr[q] > 0.f;
          if (!pos) sa[q] += pr[q] * dy[q];
          dy[q] = pos ? dy[q] : galpha[q] * dy[q];
        }
        v = Unit16<bf16>::pack(dy);
        if (do_part) {  // dbias sums dYpre before its rounding, as rdn_prelu_bwd does
#pragma unroll
          for (int q = 0; q < VEC; ++q) sb[q] += dy[q];
        }
      }
      *(u32x4*)(dyl + dlds(it)) = v;
    }
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      if (it + 1 == H_IT && tid + it * NT >= H_UNITS) continue;
      *(u32x4*)(hal + (HLIN ? (tid + it * NT) * 16 : hlds[HLIN ? 0 : it])) = hreg[it];
    }
  };

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // lane (g, q = li>>2, pp = li&3) supplies pixels {4g+q, 16+4g+q} of each 32-pixel
  // k-step and columns 4pp..4pp+3 of each 16-wide tile (ds_read_b64_tr_b16)
  const int q = li >> 2, pp = li & 3;
  const unsigned char* const pa = dyl + (4 * g + q) * DROW + 4 * pp * 2;
  const unsigned char* const pb = hal + (4 * g + q) * HROW;
  int boff[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int c = (wave + 4 * j) * 16 + 4 * pp;
    const int cc = c < NCOL ? c : 0;          // padded columns: valid reads, never stored
    const int tp = cc / CK, ci = cc - (cc / CK) * CK;
    boff[j] = ((tp / 3) * (TW + 2) + tp % 3) * HROW + ci * 2;
  }

  auto compute_tile = [&]() {
    __builtin_amdgcn_sched_barrier(0);   // keep each tile's fragment reads inside its own phase
#pragma unroll
    for (int ks = 0; ks < TP / 32; ++ks) {
      bf16x8 af[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, pa + (ks * 32) * DROW + i * 32));
        const i16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, pa + (ks * 32 + 16) * DROW + i * 32));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        if (wave + 4 * j >= NT_ALL) continue;
        const unsigned char* b = pb + boff[j] + ks * 2 * (TW + 2) * HROW;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b + (TW + 2) * HROW));
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
      }
    }
  };

  u32x4 dA[D_IT], gA[GD], hA[H_IT];
  // one tile in flight: load t+1 during tile t's MFMAs
  if (t_beg < t_end) {
    load_tile(t_beg, dA, gA, hA);
    store_tile(dA, gA, hA);
  }
  __syncthreads();
  for (int t = t_beg; t < t_end; ++t) {
    if (t + 1 < t_end) load_tile(t + 1, dA, gA, hA);
    compute_tile();
    __syncthreads();
    if (t + 1 < t_end) {
      store_tile(dA, gA, hA);
      __syncthreads();
    }
  }

  if constexpr (GATE) {
    if (do_part) {
      float* red = (float*)lds;  // the tile loop ended with a barrier
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        red[tid * VEC + k] = sa[k];
        red[NT * VEC + tid * VEC + k] = sb[k];
      }
      __syncthreads();
      if (tid < BM) {
        const int cg = tid / VEC, k = tid % VEC;
        float a = 0.f, b = 0.f;
        for (int r = 0; r < NT / DU; ++r) {
          a += red[(r * DU + cg) * VEC + k];
          b += red[NT * VEC + (r * DU + cg) * VEC + k];
        }
        const int m = m0 + tid;
        if (m < d.mdim) {
          d.part[((int64_t)bz * 2 + 0) * d.mdim + m] = a;
          d.part[((int64_t)bz * 2 + 1) * d.mdim + m] = b;
        }
      }
    }
  }
  // D[m][n]: row = g*4 + e (output channel), col = li (tile column)
  const int ncol_all = 9 * d.ndim;
  float* __restrict__ ws = d.ws + (int64_t)bz * d.mdim * ncol_all;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wave + 4 * j;
    const int c = nt * 16 + li;
    if (nt >= NT_ALL || c >= NCOL) continue;
    const int tp = c / CK, ci = c - tp * CK;
    const int col = tp * d.ndim + c0 + ci;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + i * 16 + g * 4 + e;
        if (m < d.mdim) ws[(int64_t)m * ncol_all + col] = acc[i][j][e];
      }
  }
}

struct Plan { int bm, ck, rows, glds, mtiles, chunks, tiles_x, tiles_y, ntiles, tpb, splits, chunks_rows; };

Plan plan(const rdn_wgrad_desc* d) {
  Plan p;
  p.bm = d->mdim <= 16 ? 16 : d->mdim <= 32 ? 32 : 64;
  int ck = rdn_conv3_chunk_pow2(d->ndim, d->dtype == RDN_BF16 ? 64 : 32);
  const int cap = d->dtype == RDN_BF16 ? (p.bm <= 32 ? 64 : 32) : 32;
  while (ck > cap) ck >>= 1;
  p.ck = ck;
  p.rows = 0;
  if (d->dtype == RDN_BF16) {
    // rows kernel: the widest channel group whose accumulators fit (BM x 9 CK per block)
    // accumulator budget BM x CK <= 2560: two blocks per CU (measured r01: a
    // 4096 budget at one block per CU, and 128-channel blocks, were slower)
    const int maxacc = 2560, bm = p.bm;
    static const int cands[] = {96, 80, 64, 48, 32, 16, 8};
    for (int c : cands)
      if (d->ndim % c == 0 && c * bm <= maxacc) { p.ck = c; p.rows = 1; p.bm = bm; break; }
  }
  p.chunks_rows = d->ndim / p.ck;   // the PReLU-gate fusion decision (rdn_wgrad_chunks) is made on these
  p.glds = 0;
  p.tiles_x = (d->w + TW - 1) / TW;
  p.tiles_y = (d->h + TH - 1) / TH;
  p.ntiles = d->n * p.tiles_x * p.tiles_y;
  // the LDS-DMA pipelined kernel (wgrad3_glds.hip), one block per CU: multi-chunk
  // launches (no gate) and the single-chunk level-0/1 ones (gate fused)
  if (p.rows && rdn_wgrad3_glds_pick(d, p.chunks_rows == 1, &p.bm, &p.ck)) {
    p.glds = 1;
    p.mtiles = (d->mdim + p.bm - 1) / p.bm;
    p.chunks = d->ndim / p.ck;
    const int base = p.mtiles * p.chunks;
    // blocks per launch: 128 of the 256 CUs, leaving room beside the dgrad chain;
    // step A/B (3 interleaved rounds, same box): 128: 1483, 192: 1506, 256: 1499,
    // 512: 1416 img/s (past 256 the 1-per-CU blocks run in two waves); re-measured in
    // r03 (profiles/r03_v10_wglds_blocks_ab.txt): 96: 1633, 128: 1698, 160: 1714,
    // 192: 1714, 256: 1687; round 4, after the fused layers' work moved onto the
    // compute stream (gate-out, batched reduce): 192: 1767 / 1991, 160: 1777 / 1997,
    // 128: 1777 / 2011 img/s B16 / B32, then 128: 1764 / 1975, 112: 1759 / 1957,
    // 96: 1730 / 1927 (profiles/r04_v28_wglds_blocks_ab.txt, r04_v29_*).  RDN_WGLDS_BLOCKS
    static const int gtarget = [] {
      const char* e = getenv("RDN_WGLDS_BLOCKS");
      const int v = e ? atoi(e) : 0;
      return v > 0 ? v : 128;
    }();
    int s = d->splits > 0 ? d->splits : gtarget / base;
    const int maxs = (p.ntiles + 1) / 2;                             // >= 2 tiles per block
    if (s > maxs) s = maxs;
    if (s < 1) s = 1;
    p.tpb = (p.ntiles + s - 1) / s;
    p.splits = s;
    return p;
  }
  p.mtiles = (d->mdim + p.bm - 1) / p.bm;
  p.chunks = d->ndim / p.ck;
  const int base = p.mtiles * p.chunks;
  // blocks per launch: one per CU.  The weight gradients run on the side stream
  // beside the dgrad chain, where fewer, longer blocks (and half the split-K slab
  // bytes) won: whole step 1342 (512) -> 1362 (256) img/s; 128: 1165, 192: 1302,
  // 384: 1355, 1024: 1311
  constexpr int target = 256;
  int s = d->splits > 0 ? d->splits : (target + base - 1) / base;
  const int maxs = (p.ntiles + 3) / 4;                             // >= 4 tiles per block
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  p.tpb = (p.ntiles + s - 1) / s;
  p.splits = s;  // blocks past the last tile write zero slabs, so any s is exact
  return p;
}

template <typename T, int BM, int CK>
int launch_w(const rdn_wgrad_desc* d, const Plan& p, hipStream_t st) {
  dim3 grid(p.mtiles, p.chunks, p.splits);
  RDN_PROBE("wgrad3_halo_kernel<%s,%d,%d%s>", rdn_tname<T>(), BM, CK, d->a_gate ? ",gate" : "");
  if (d->a_gate)
    wgrad3_halo_kernel<T, BM, CK, true><<<grid, NT, 0, st>>>(*d, p.tiles_x, p.tiles_y, p.ntiles, p.tpb);
  else
    wgrad3_halo_kernel<T, BM, CK, false><<<grid, NT, 0, st>>>(*d, p.tiles_x, p.tiles_y, p.ntiles, p.tpb);
  return rdn_check_launch("rdn_conv_wgrad(conv3)");
}

template <int BM, int CK>
int launch_rows(const rdn_wgrad_desc* d, const Plan& p, hipStream_t st) {
  if constexpr (CK * BM > 4096) {
    rdn_set_error("rdn_conv_wgrad(conv3): rows kernel BM=%d CK=%d", BM, CK);
    return RDN_E_SHAPE;
  } else {
    dim3 grid(p.mtiles * p.chunks * p.splits);
    RDN_PROBE("wgrad3_rows_kernel<bf16,%d,%d%s>", BM, CK, d->a_gate ? ",gate" : "");
    if (d->a_gate)
      wgrad3_rows_kernel<BM, CK, true><<<grid, NT, 0, st>>>(*d, p.tiles_x, p.tiles_y, p.ntiles, p.tpb);
    else
      wgrad3_rows_kernel<BM, CK, false><<<grid, NT, 0, st>>>(*d, p.tiles_x, p.tiles_y, p.ntiles, p.tpb);
    return rdn_check_launch("rdn_conv_wgrad(conv3 rows)");
  }
}

template <int BM>
int launch_rows_ck(const rdn_wgrad_desc* d, const Plan& p, hipStream_t st) {
  switch (p.ck) {
    case 96: return launch_rows<BM, 96>(d, p, st);
    case 80: return launch_rows<BM, 80>(d, p, st);
    case 64: return launch_rows<BM, 64>(d, p, st);
    case 48: return launch_rows<BM, 48>(d, p, st);
    case 32: return launch_rows<BM, 32>(d, p, st);
    case 16: return launch_rows<BM, 16>(d, p, st);
    case 8: return launch_rows<BM, 8>(d, p, st);
  }
  rdn_set_error("rdn_conv_wgrad(conv3): bad chunk %d", p.ck);
  return RDN_E_SHAPE;
}

template <typename T, int BM>
int launch_ck(const rdn_wgrad_desc* d, const Plan& p, hipStream_t st) {
  switch (p.ck) {
    case 64: if constexpr (sizeof(T) == 2 && BM <= 32) return launch_w<T, BM, 64>(d, p, st); break;
    case 32: return launch_w<T, BM, 32>(d, p, st);
    case 16: return launch_w<T, BM, 16>(d, p, st);
    case 8: return launch_w<T, BM, 8>(d, p, st);
  }
  rdn_set_error("rdn_conv_wgrad(conv3): bad chunk %d", p.ck);
  return RDN_E_SHAPE;
}

}  // namespace

int rdn_wgrad3_splits(const rdn_wgrad_desc* d) { return plan(d).splits; }
int rdn_wgrad3_chunks(const rdn_wgrad_desc* d) { return plan(d).chunks_rows; }

int rdn_wgrad3_launch(const rdn_wgrad_desc* d, hipStream_t st) {
  const Plan p = plan(d);
  if (p.ck <= 0) { rdn_set_error("rdn_conv_wgrad(conv3): ndim=%d", d->ndim); return RDN_E_SHAPE; }
  if (p.glds)
    return rdn_wgrad3_glds_launch(d, p.bm, p.ck, p.mtiles * p.chunks * p.splits, p.tiles_x, p.tiles_y, p.ntiles,
                                  p.tpb, st);
  if (p.rows) {
    if (p.bm == 16) return launch_rows_ck<16>(d, p, st);
    if (p.bm == 32) return launch_rows_ck<32>(d, p, st);
    return launch_rows_ck<64>(d, p, st);
  }
  if (d->dtype == RDN_BF16) {
    if (p.bm == 16) return launch_ck<bf16, 16>(d, p, st);
    if (p.bm == 32) return launch_ck<bf16, 32>(d, p, st);
    return launch_ck<bf16, 64>(d, p, st);
  }
  if (p.bm == 16) return launch_ck<float, 16>(d, p, st);
  if (p.bm == 32) return launch_ck<float, 32>(d, p, st);
  return launch_ck<float, 64>(d, p, st);
}
