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
          v = *(const u32x4*)(A + pix * d.a_ps + d.a_c0 + m);
          if constexpr (GATE) gv = *(const u32x4*)(G + pix * d.a_gate_ps + m);
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
          v = *(const u32x4*)(Bx + (((int64_t)nimg * H + yy) * W + xx) * d.b_ps + d.b_c0 + c0 + cu * VEC);
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

struct Plan { int bm, ck, mtiles, chunks, tiles_x, tiles_y, ntiles, tpb, splits; };

Plan plan(const rdn_wgrad_desc* d) {
  Plan p;
  p.bm = d->mdim <= 16 ? 16 : d->mdim <= 32 ? 32 : 64;
  int ck = rdn_conv3_chunk_pow2(d->ndim, d->dtype == RDN_BF16 ? 64 : 32);
  const int cap = d->dtype == RDN_BF16 ? (p.bm <= 32 ? 64 : 32) : 32;
  while (ck > cap) ck >>= 1;
  p.ck = ck;
  p.mtiles = (d->mdim + p.bm - 1) / p.bm;
  p.chunks = d->ndim / ck;
  p.tiles_x = (d->w + TW - 1) / TW;
  p.tiles_y = (d->h + TH - 1) / TH;
  p.ntiles = d->n * p.tiles_x * p.tiles_y;
  const int base = p.mtiles * p.chunks;
  int s = d->splits > 0 ? d->splits : (512 + base - 1) / base;     // ~2 blocks per CU
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
  if (d->a_gate)
    wgrad3_halo_kernel<T, BM, CK, true><<<grid, NT, 0, st>>>(*d, p.tiles_x, p.tiles_y, p.ntiles, p.tpb);
  else
    wgrad3_halo_kernel<T, BM, CK, false><<<grid, NT, 0, st>>>(*d, p.tiles_x, p.tiles_y, p.ntiles, p.tpb);
  return rdn_check_launch("rdn_conv_wgrad(conv3)");
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
int rdn_wgrad3_chunks(const rdn_wgrad_desc* d) { return plan(d).chunks; }

int rdn_wgrad3_launch(const rdn_wgrad_desc* d, hipStream_t st) {
  const Plan p = plan(d);
  if (p.ck <= 0) { rdn_set_error("rdn_conv_wgrad(conv3): ndim=%d", d->ndim); return RDN_E_SHAPE; }
  if (d->dtype == RDN_BF16) {
    if (p.bm == 16) return launch_ck<bf16, 16>(d, p, st);
    if (p.bm == 32) return launch_ck<bf16, 32>(d, p, st);
    return launch_ck<bf16, 64>(d, p, st);
  }
  if (p.bm == 16) return launch_ck<float, 16>(d, p, st);
  if (p.bm == 32) return launch_ck<float, 32>(d, p, st);
  return launch_ck<float, 64>(d, p, st);
}
